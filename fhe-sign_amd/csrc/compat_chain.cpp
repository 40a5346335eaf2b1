// compat_chain.cpp -- the reference's BigUintFHE mul limbs (src/biguint.rs:194-265, lost carries
// included: SURVEY F7) as a carry-count chain of one lookup level per limb.
//
// The reference's step (i, j) adds P = a_i b_j into the 96-bit window of limbs idx = i + j .. idx + 2
// and drops the carry out of its top (:234-249).  Seen from one limb l, the steps touching it come in
// step order with one of three roles:
//   BOT (idx = l):     adds lo(P), no carry in; its crossing (carry out) goes to limb l + 1
//   MID (idx = l - 1): adds hi(P) + the carry from l - 1; crossing goes to l + 1 (dropped at the top limb)
//   TOP (idx = l - 2): adds the carry from l - 1 only; crossing dropped
// With K(t) = the known addends of l so far and k(t) = the carries into l so far, the crossings so
// far are C(t) = floor((K + k) / 2^32) = H(t) + beta(t), H = floor(K / 2^32) and
// beta = [K mod 2^32 + k >= 2^32].  For min(la, lb) <= 8, k <= 15, so beta = [k - g - 1 >= 0] with
// g = 15 - near * (K mod 16), near = [K mod 2^32 >= 2^32 - 16]: K only enters through g and H,
// which are prefix sums of product halves -- off the chain, throughput work.  The carries into
// l + 1 up to step s telescope over l's touches:
//   k_{l+1}(s) = H_l(u) + beta_l(u) - sum_{TOP touches w <= s} (beta_l(w) - beta_l(prev w)),
// u = l's last touch at or before s (a TOP touch adds nothing to K, so H cancels there).  So every
// beta of limb l + 1 is ONE lookup of a linear combination of limb l's betas: the chain is one level
// per limb (16 for 8 x 8 limbs), where the window adds of the dependency-wave form took 4 levels per
// wave (36 waves).  The final limb is (K_l(last) + k_l(final)) mod 2^32.  Integer model, checked
// against the reference's limb loop: tools/compat_chain_sim.py.
//
// Encodings (raw PbsItems, radix.h): beta is produced by a sign lookup -- a constant +1/2-step LUT,
// whose negacyclic half gives -1/2 for inputs in [-16, 0) -- so the block holds s = beta - 1/2 and
// every linear use of it adds the 1/2 back as a half-step constant.  The sign input k - g - 1 lies in
// [-16, 14].
#include <chrono>
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "biguint.h"

namespace fhe {

namespace {

std::vector<uint32_t> table(uint32_t (*f)(uint32_t)) {
    std::vector<uint32_t> t(16);
    for (uint32_t v = 0; v < 16; ++v) t[v] = f(v) & 15u;
    return t;
}

PbsItem item(const std::vector<Term>& terms, std::vector<uint32_t> tab, uint32_t cst = 0) {
    PbsItem it;
    it.terms = terms;
    it.table = std::move(tab);
    it.cst = cst;
    return it;
}

// raw item: outputs f(v) (message steps, integer) for v in [0, 16)
PbsItem raw_item(const std::vector<Term>& terms, int32_t half_cst, uint32_t (*f)(uint32_t), uint32_t degree) {
    PbsItem it;
    it.raw = true;
    it.terms = terms;
    it.half_cst = half_cst;
    it.half_table.resize(16);
    for (uint32_t v = 0; v < 16; ++v) it.half_table[v] = 2 * (int32_t)f(v);
    it.raw_degree = degree;
    return it;
}

// sign item: s = +1/2 if the input is in [0, 16), -1/2 if in [-16, 0)
PbsItem sign_item(const std::vector<Term>& terms, int32_t half_cst) {
    PbsItem it;
    it.raw = true;
    it.terms = terms;
    it.half_cst = half_cst;
    it.half_table.assign(16, 1);
    it.raw_degree = 1;
    return it;
}

}  // namespace

// g = 15 - near * (K mod 16) of each prefix, from its 16 columns (column 0 one block <= 3, columns
// 1..15 two blocks <= 3 each: v_m <= 6).  near = [K mod 2^32 >= 2^32 - 16] = [the resolved blocks
// r_2..r_15 all equal 3], r_m = (v_m + c_m) mod 4, c_{m+1} = [v_m + c_m >= 4], c_1 = 0 (v_0 <= 3).
// r_m = 3 means v_m + c_m in {3, 7}; a carry cannot start at a block that resolves to 3 (v_m = 7 is
// out of range), so while every block below m resolves to 3, c_m = [v_{m-1} >= 4] (for m = 2 that
// is the exact carry [v_1 >= 4]; above, v_{m-1} + c_{m-1} = 7 needs v_{m-1} = 6).  The local
// indicators e_m = [(v_m + [v_{m-1} >= 4]) mod 4 == 3] therefore agree with [r_m == 3] at every block
// up to the first one that is not 3, and near = AND of e_2..e_15 is exact.  (A bare [v_m == 3] for
// m >= 3 is not: v_2 = 6 with c_2 = 1 resolves to 3 and carries into block 3.)  Five levels:
// [v_m >= 4] and v_1 mod 4; the e_m; near; the two ANDs with K mod 16; g.
Blocks compat_chain_g(Engine& e, const std::vector<const std::vector<Blocks>*>& P) {
    static const auto GE4 = table([](uint32_t v) { return v >= 4 ? 1u : 0u; });
    static const auto MOD4 = table([](uint32_t v) { return v & 3u; });
    static const auto MOD4_EQ3 = table([](uint32_t v) { return (v & 3u) == 3 ? 1u : 0u; });
    static const auto ID = table([](uint32_t v) { return v; });
    static const auto AND_ = [] {
        std::vector<uint32_t> t(16);
        for (uint32_t v = 0; v < 16; ++v) t[v] = (v >> 2) ? (v & 3u) : 0u;
        return t;
    }();
    auto terms = [](const Blocks& col) {
        std::vector<Term> t;
        for (const Block& b : col) t.push_back({b, 1});
        return t;
    };
    const size_t np = P.size();
    constexpr uint32_t kGe = kLimbBlocks - 2;  // [v_m >= 4], m = 1..14
    std::vector<PbsItem> items;
    for (const auto* cols : P) {
        engine_check(cols->size() == kLimbBlocks && (*cols)[0].size() == 1, "compat chain: prefix column shape");
        for (uint32_t m = 1; m + 1 < kLimbBlocks; ++m) items.push_back(item(terms((*cols)[m]), GE4));
        items.push_back(item(terms((*cols)[1]), MOD4));
    }
    Blocks l1 = e.run(items);
    items.clear();
    for (size_t k = 0; k < np; ++k) {
        const auto& cols = *P[k];
        for (uint32_t m = 2; m < kLimbBlocks; ++m) {
            std::vector<Term> t = terms(cols[m]);
            t.push_back({l1[k * (kGe + 1) + (m - 2)], 1});  // [v_{m-1} >= 4]
            items.push_back(item(t, MOD4_EQ3));
        }
    }
    Blocks ind = e.run(items);
    // near = all 14 indicators (raw: a 14-term input)
    items.clear();
    for (size_t k = 0; k < np; ++k) {
        std::vector<Term> t;
        for (uint32_t m = 2; m < kLimbBlocks; ++m) t.push_back({ind[k * (kLimbBlocks - 2) + (m - 2)], 1});
        items.push_back(raw_item(t, 0, [](uint32_t v) { return v == kLimbBlocks - 2 ? 1u : 0u; }, 1));
    }
    Blocks near = e.run(items);
    // g = 15 - near * (4 b1 + b0), b1 = v_1 mod 4, b0 = column 0's single block
    items.clear();
    for (size_t k = 0; k < np; ++k) {
        const Block& b1 = l1[k * (kGe + 1) + kGe];
        items.push_back(item({{near[k], 4}, {b1, 1}}, AND_));
        items.push_back(item({{near[k], 4}, {(*P[k])[0][0], 1}}, AND_));
    }
    Blocks outs = e.run(items);
    items.clear();
    for (size_t k = 0; k < np; ++k) items.push_back(item({{outs[2 * k], -4}, {outs[2 * k + 1], -1}}, ID, 15));
    return e.run(items);
}

namespace {

enum Role { kBot, kMid, kTop };

struct Touch {
    size_t step;   // reference step index (i outer, j inner)
    size_t prod;   // product index i * lb + j
    Role role;
    int prefix;    // index into the limb's prefixes (addends so far - 1), -1 before the first addend
};

// A linear combination with half-step constant (the carry counts k)
struct Lin {
    std::vector<Term> terms;
    int32_t half = 0;  // constant, half message steps
};

}  // namespace

bool compat_chain_applies(size_t la, size_t lb) { return std::min(la, lb) >= 2 && std::min(la, lb) <= 8; }

BigUint compat_chain_mul(Engine& e, const BigUint& A, const BigUint& B) {
    const size_t la = A.digits.size(), lb = B.digits.size(), L = la + lb;
    // FHE_DEBUG=chain (diagnostic, dry runs): flush and print the bootstrap count after each phase;
    // chain-host: host time only, no flush
    const bool phases = debug().chain || debug().chain_host;
    const auto t0 = std::chrono::steady_clock::now();
    auto phase = [&](const char* what) {
        if (!phases) return;
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (debug().chain_host) {  // host time only
            fprintf(stderr, "[compat chain] %-28s host %7.1f ms\n", what, ms);
            return;
        }
        e.flush();
        fprintf(stderr, "[compat chain] %-28s %8llu PBS %4llu levels  host %7.1f ms\n", what,
                (unsigned long long)e.pbs_count, (unsigned long long)e.levels, ms);
    };
    engine_check(compat_chain_applies(la, lb), "compat chain: limb counts");
    // ---- the 64-bit products a_i * b_j: one batched multiplication, columns compressed but not
    // propagated (each <= 6 over <= 3 blocks; exact, as the products fit 32 columns).  Split at the
    // limb boundary: lo_cs = columns 0..15 = lo(P) + 2^32 c_P, hi_cs = columns 16..31 = hi(P) - c_P,
    // c_P = the carry out of column 15 (a bit): only c_P is resolved per product, not the product.
    std::vector<Radix> a64(la), b64(lb);
    for (size_t i = 0; i < la; ++i) a64[i] = radix_resize(A.digits[i], 2 * kLimbBlocks);
    for (size_t j = 0; j < lb; ++j) b64[j] = radix_resize(B.digits[j], 2 * kLimbBlocks);
    std::vector<std::pair<const Radix*, const Radix*>> ops;
    for (size_t i = 0; i < la; ++i)
        for (size_t j = 0; j < lb; ++j) ops.push_back({&a64[i], &b64[j]});
    // (Karatsuba-split products come with a 33rd column and a public excess q: their columns sum to
    // P + q 2^64, i.e. hi(P) = hi_cs + c_P + 2^32 (column 32 - q); a MID addend takes column 32 - q
    // into the limb's overflow O below)
    std::vector<int64_t> excess;
    // the high half (hi(P) columns) is read only by the prefix sums, whose inputs take a previous prefix
    // column (<= 6) plus the product column: <= 9 there suffices
    constexpr uint32_t hi_lim = 9;
    std::vector<std::vector<Blocks>> PC = radix_mul_many_columns(e, ops, 2 * kLimbBlocks, &excess, kLimbBlocks, hi_lim);
    phase("product columns");
    {
        // entries must be fresh-noise blocks for the accumulation's noise budget (lazy multiples of a
        // public block -- only from trivially encrypted limbs -- are refreshed)
        static const auto ID = table([](uint32_t v) { return v; });
        std::vector<PbsItem> items;
        std::vector<Block*> at;
        for (auto& cols : PC)
            for (auto& c : cols)
                for (Block& b : c)
                    if (!b.trivial() && (b.noise > 1 || (b.lazy() && b.lin->size() > 1))) {
                        items.push_back(item({{b, 1}}, ID));
                        at.push_back(&b);
                    }
        if (!items.empty()) {
            Blocks outs = e.run(items);
            for (size_t k = 0; k < outs.size(); ++k) *at[k] = outs[k];
        }
    }
    phase("refresh");
    Blocks cP;
    {
        std::vector<std::vector<Blocks>> lo(PC.size());
        for (size_t k = 0; k < PC.size(); ++k) lo[k].assign(PC[k].begin(), PC[k].begin() + kLimbBlocks);
        cP = radix_carry_outs(e, lo);
    }
    phase("products");

    // ---- touches per limb
    std::vector<std::vector<Touch>> T(L);
    for (size_t i = 0, s = 0; i < la; ++i)
        for (size_t j = 0; j < lb; ++j, ++s) {
            const size_t idx = i + j;
            T[idx].push_back({s, s, kBot, -1});
            T[idx + 1].push_back({s, s, kMid, -1});
            if (idx + 2 < L) T[idx + 2].push_back({s, s, kTop, -1});
        }
    // ---- prefix sums of each limb's addends, K_acc(p) = K(p) + 2^32 * (c_P of the BOT addends so far):
    // 16 columns kept at <= 2 entries (lo <= 3 + incoming hi <= 2; position 0 lo only) by one
    // compression per addend (a MID addend hi_cs brings its c_P along at column 0), the carries out of
    // column 15 in a small-integer block O = 1 + sum(hi_15) - sum(c_P of BOT addends), so that
    // H = floor(K / 2^32) = O - 1 + c1, c1 = the carry out of the 16 columns.  O stays in [0, 15]:
    // O - 1 = H - c1 >= -1 and H <= 14.
    struct Prefix {
        std::vector<Blocks> cols;  // 16 columns
        Block O;                   // biased overflow (above)
        Block c1;                  // carry out of the 16 columns
        Block g;                   // 15 - near * (K mod 16)
    };
    std::vector<std::vector<Prefix>> PF(L);
    {
        static const auto MOD4 = table([](uint32_t v) { return v & 3u; });
        static const auto DIV4 = table([](uint32_t v) { return v >> 2; });
        // every limb advances one addend per round (rounds run independently in the engine graph;
        // the grouping only batches the host work)
        std::vector<size_t> next(L, 0);
        std::vector<std::vector<std::pair<size_t, int>>> adds(L);  // (product, half: 0 lo / 1 hi)
        for (size_t l = 0; l < L; ++l)
            for (Touch& t : T[l]) {
                if (t.role == kBot) adds[l].push_back({t.prod, 0});
                if (t.role == kMid) adds[l].push_back({t.prod, 1});
                t.prefix = (int)adds[l].size() - 1;
            }
        for (size_t l = 0; l < L; ++l) PF[l].resize(adds[l].size());
        const Block kBias = Block::make_trivial(1);
        for (bool more = true; more;) {
            more = false;
            std::vector<PbsItem> items;
            struct Dst {
                size_t l, p;
                int col;  // 0..15: lo of that column; 16 + c: hi of column c
            };
            std::vector<Dst> dst;
            for (size_t l = 0; l < L; ++l) {
                const size_t p = next[l];
                if (p >= adds[l].size()) continue;
                more = true;
                next[l]++;
                const auto& pc = PC[adds[l][p].first];
                const bool hi = adds[l][p].second != 0;
                const uint32_t off = hi ? kLimbBlocks : 0;
                for (uint32_t m = 0; m < kLimbBlocks; ++m) {
                    std::vector<Term> t;
                    if (p > 0)
                        for (const Block& b : PF[l][p - 1].cols[m]) t.push_back({b, 1});
                    for (const Block& b : pc[off + m]) t.push_back({b, 1});
                    if (hi && m == 0) t.push_back({cP[adds[l][p].first], 1});
                    items.push_back(item(t, MOD4));
                    dst.push_back({l, p, (int)m});
                    items.push_back(item(t, DIV4));
                    dst.push_back({l, p, 16 + (int)m});
                }
            }
            if (items.empty()) continue;
            Blocks outs = e.run(items);
            // assemble the new columns, then the overflow update (O + hi_15 - [BOT] c_P)
            std::vector<PbsItem> oitems;
            std::vector<std::pair<size_t, size_t>> odst;
            for (size_t k = 0; k < outs.size(); ++k) {
                Prefix& x = PF[dst[k].l][dst[k].p];
                if (x.cols.empty()) x.cols.assign(kLimbBlocks, {});
                const int c = dst[k].col;
                if (c < 16) {
                    x.cols[c].push_back(outs[k]);
                } else if (c - 16 + 1 < (int)kLimbBlocks) {
                    x.cols[c - 16 + 1].push_back(outs[k]);
                } else {  // hi of column 15 -> overflow
                    const size_t l = dst[k].l, p = dst[k].p;
                    const Block& O0 = p ? PF[l][p - 1].O : kBias;
                    std::vector<Term> t{{O0, 1}, {outs[k], 1}};
                    int32_t half = 0;
                    const size_t prod = adds[l][p].first;
                    if (adds[l][p].second == 0) {
                        t.push_back({cP[prod], -1});
                    } else if (PC[prod].size() > 2 * kLimbBlocks) {
                        for (const Block& b : PC[prod][2 * kLimbBlocks]) t.push_back({b, 1});
                        half = -2 * (int32_t)excess[prod];
                    }
                    oitems.push_back(raw_item(t, half, [](uint32_t v) { return v; }, 15));
                    odst.push_back({l, p});
                }
            }
            Blocks os = e.run(oitems);
            for (size_t k = 0; k < os.size(); ++k) PF[odst[k].first][odst[k].second].O = os[k];
        }
    }
    phase("prefix sums");
    // ---- per prefix: c1 (carry out of the 16 columns) and g
    {
        std::vector<std::vector<Blocks>> probs;
        std::vector<std::pair<size_t, size_t>> where;
        for (size_t l = 0; l < L; ++l)
            for (size_t p = 0; p < PF[l].size(); ++p) {
                probs.push_back(PF[l][p].cols);
                where.push_back({l, p});
            }
        Blocks c1 = radix_carry_outs(e, probs);
        for (size_t k = 0; k < c1.size(); ++k) PF[where[k].first][where[k].second].c1 = c1[k];
        phase("carry outs c1");
        std::vector<const std::vector<Blocks>*> cols;
        for (auto& w : where) cols.push_back(&PF[w.first][w.second].cols);
        Blocks g = compat_chain_g(e, cols);
        for (size_t k = 0; k < where.size(); ++k) PF[where[k].first][where[k].second].g = g[k];
    }

    phase("g");
    // ---- the chain: s = beta - 1/2 of every touch, limb by limb
    std::vector<std::vector<Block>> S(L);  // S[l][touch]
    const Block kNeg = Block::make_trivial(0);  // marker: beta == 0 known (s = -1/2)
    std::vector<std::vector<bool>> s_known0(L);
    // k_{l}(step) as a linear combination of limb l - 1's quantities
    auto k_of = [&](size_t l, size_t step, Lin* k) -> bool {  // false: k == 0 structurally
        k->terms.clear();
        k->half = 0;
        if (l == 0) return false;
        const auto& prev = T[l - 1];
        int u = -1;
        for (size_t m = 0; m < prev.size(); ++m)
            if (prev[m].step <= step) u = (int)m;
        if (u < 0) return false;
        auto add_s = [&](size_t m, int32_t c) {  // c * beta_{l-1}(m) = c * (s + 1/2)
            k->half += c;
            if (s_known0[l - 1][m])
                k->half += -c;  // s = -1/2 exactly: c * s = -c/2
            else
                k->terms.push_back({S[l - 1][m], c});
        };
        const Prefix* hp = prev[u].prefix >= 0 ? &PF[l - 1][prev[u].prefix] : nullptr;
        if (hp) {  // H = O - 1 + c1
            k->terms.push_back({hp->O, 1});
            k->terms.push_back({hp->c1, 1});
            k->half -= 2;
        }
        add_s(u, 1);
        for (size_t m = 0; m < prev.size() && prev[m].step <= step; ++m)
            if (prev[m].role == kTop) {
                add_s(m, -1);
                if (m > 0) add_s(m - 1, 1);  // a first touch has no predecessor: C = 0 before it
            }
        // fold trivial terms (publicly known values: the host-only CPU runs have nothing else)
        std::vector<Term> live;
        int32_t cst2 = k->half;
        for (const Term& t : k->terms) {
            if (t.b.trivial())
                cst2 += t.coef * (int32_t)trivial_half2(t.b);
            else
                live.push_back(t);
        }
        k->terms = live;
        k->half = cst2;
        return !(live.empty() && cst2 == 0);  // false: k == 0 known
    };
    for (size_t l = 0; l < L; ++l) {
        S[l].assign(T[l].size(), kNeg);
        s_known0[l].assign(T[l].size(), true);
        std::vector<PbsItem> items;
        std::vector<size_t> at;
        for (size_t m = 0; m < T[l].size(); ++m) {
            Lin k;
            if (!k_of(l, T[l][m].step, &k)) continue;  // no carry in yet: beta = 0
            const int pf = T[l][m].prefix;
            if (pf < 0) continue;  // no addend yet: K = 0, so g = 15 > k - 1 and beta = 0
            std::vector<Term> t = k.terms;
            t.push_back({PF[l][pf].g, -1});
            items.push_back(sign_item(t, k.half - 2));  // k - g - 1
            at.push_back(m);
        }
        if (items.empty()) continue;
        Blocks outs = e.run(items);
        for (size_t q = 0; q < at.size(); ++q) {
            S[l][at[q]] = outs[q];
            s_known0[l][at[q]] = false;
        }
        if (phases) {
            int32_t dmax = 0, gmax = 0;
            for (size_t q = 0; q < at.size(); ++q) {
                dmax = std::max(dmax, e.depth_of(outs[q]));
                gmax = std::max(gmax, e.depth_of(PF[l][T[l][at[q]].prefix].g));
            }
            fprintf(stderr, "[compat chain] limb %2zu: %zu signs, depth %d (its g: %d)\n", l, at.size(), dmax, gmax);
        }
    }

    phase("chain");
    // ---- final limbs: (K_l(last) + k_l(final)) mod 2^32
    BigUint out;
    out.digits.resize(L);
    {
        // K_l(last) mod 2^32, canonical
        std::vector<Radix> X(L);
        for (size_t l = 0; l < L; ++l) X[l] = radix_propagate_columns(e, PF[l].back().cols, kLimbBlocks);
        std::vector<Lin> kf(L);
        std::vector<bool> has_k(L);
        for (size_t l = 0; l < L; ++l) has_k[l] = k_of(l, (size_t)-1, &kf[l]);
        static const auto EQ3 = table([](uint32_t v) { return v == 3 ? 1u : 0u; });
        static const auto ID = table([](uint32_t v) { return v; });
        // indicators [x_m == 3], m = 2..14, and y = x_0 + 4 x_1
        std::vector<Blocks> ind(L);
        std::vector<Block> y(L);
        {
            std::vector<PbsItem> items;
            for (size_t l = 0; l < L; ++l) {
                if (!has_k[l]) continue;
                for (uint32_t m = 2; m + 1 < kLimbBlocks; ++m) items.push_back(item({{X[l].blocks[m], 1}}, EQ3));
                items.push_back(item({{X[l].blocks[1], 4}, {X[l].blocks[0], 1}}, ID));
            }
            Blocks outs = e.run(items);
            size_t o = 0;
            for (size_t l = 0; l < L; ++l) {
                if (!has_k[l]) continue;
                ind[l].assign(outs.begin() + o, outs.begin() + o + (kLimbBlocks - 3));
                o += kLimbBlocks - 3;
                y[l] = outs[o++];
            }
        }
        // z_m = x_m + 4 [x_2..x_{m-1} all 3], m = 2..15 (m = 2: the empty AND is 1)
        std::vector<Blocks> z(L);
        {
            std::vector<PbsItem> items;
            for (size_t l = 0; l < L; ++l) {
                if (!has_k[l]) continue;
                for (uint32_t m = 3; m < kLimbBlocks; ++m) {
                    std::vector<Term> t;
                    for (uint32_t q = 2; q < m; ++q) t.push_back({ind[l][q - 2], 1});
                    const uint32_t cnt = m - 2;
                    PbsItem it;
                    it.raw = true;
                    it.terms = t;
                    it.half_table.resize(16);
                    for (uint32_t v = 0; v < 16; ++v) it.half_table[v] = v == cnt ? 2 : 0;
                    it.raw_degree = 1;
                    items.push_back(it);
                }
            }
            Blocks pm = e.run(items);
            items.clear();
            size_t o = 0;
            for (size_t l = 0; l < L; ++l) {
                if (!has_k[l]) continue;
                items.push_back(item({{X[l].blocks[2], 1}}, ID, 4));  // p_2 = 1: z_2 = x_2 + 4
                for (uint32_t m = 3; m < kLimbBlocks; ++m) items.push_back(item({{pm[o++], 4}, {X[l].blocks[m], 1}}, ID));
            }
            Blocks zs = e.run(items);
            o = 0;
            for (size_t l = 0; l < L; ++l) {
                if (!has_k[l]) continue;
                z[l].assign(zs.begin() + o, zs.begin() + o + (kLimbBlocks - 2));
                o += kLimbBlocks - 2;
            }
        }
        // tail: level 1 -- c_low = [y + k >= 16] (sign), k0 = k mod 4, k1 = k div 4
        std::vector<PbsItem> items;
        for (size_t l = 0; l < L; ++l) {
            if (!has_k[l]) continue;
            std::vector<Term> t = kf[l].terms;
            t.push_back({y[l], 1});
            items.push_back(sign_item(t, kf[l].half - 32));
            items.push_back(raw_item(kf[l].terms, kf[l].half, [](uint32_t v) { return v & 3u; }, 3));
            items.push_back(raw_item(kf[l].terms, kf[l].half, [](uint32_t v) { return v >> 2; }, 3));
        }
        Blocks t1 = e.run(items);
        // level 2: b_0, c0, b_m (m >= 2) = (x_m + [p_m and c_low]) mod 4 from z_m + 4 (s + 1/2)
        items.clear();
        static const auto SUM_MOD4 = table([](uint32_t v) { return v & 3u; });
        static const auto SUM_GE4 = table([](uint32_t v) { return v >= 4 ? 1u : 0u; });
        size_t o = 0;
        for (size_t l = 0; l < L; ++l) {
            if (!has_k[l]) continue;
            const Block &sc = t1[o], &k0 = t1[o + 1];
            o += 3;
            items.push_back(item({{X[l].blocks[0], 1}, {k0, 1}}, SUM_MOD4));
            items.push_back(item({{X[l].blocks[0], 1}, {k0, 1}}, SUM_GE4));
            for (uint32_t m = 2; m < kLimbBlocks; ++m)
                items.push_back(raw_item({{z[l][m - 2], 1}, {sc, 4}}, 4,
                                         [](uint32_t v) { return ((v & 3u) + (v >= 8 ? 1u : 0u)) & 3u; }, 3));
        }
        Blocks t2 = e.run(items);
        // level 3: b_1 = (x_1 + k1 + c0) mod 4
        items.clear();
        o = 0;
        size_t o2 = 0;
        for (size_t l = 0; l < L; ++l) {
            if (!has_k[l]) continue;
            const Block& k1 = t1[o + 2];
            o += 3;
            items.push_back(item({{X[l].blocks[1], 1}, {k1, 1}, {t2[o2 + 1], 1}}, SUM_MOD4));
            o2 += 2 + (kLimbBlocks - 2);
        }
        Blocks t3 = e.run(items);
        o2 = 0;
        size_t o3 = 0;
        for (size_t l = 0; l < L; ++l) {
            Radix r;
            if (!has_k[l]) {
                r = X[l];
            } else {
                r.blocks.resize(kLimbBlocks);
                r.blocks[0] = t2[o2];
                r.blocks[1] = t3[o3++];
                for (uint32_t m = 2; m < kLimbBlocks; ++m) r.blocks[m] = t2[o2 + 2 + (m - 2)];
                o2 += 2 + (kLimbBlocks - 2);
            }
            out.digits[l] = std::move(r);
        }
    }
    phase("final limbs");
    return out;
}

}  // namespace fhe
