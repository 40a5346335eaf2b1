"""Plaintext restatement of the reference's BigUintFHE limb semantics and BIP-340 signer.

TEST INFRASTRUCTURE ONLY (checker + golden-vector generator; never imported by fhe-sign_amd/).

Follows, line by line in meaning:
  src/biguint.rs:17-31     BigUintFHE::new  -> to_u32_digits (LSB first, [] for zero)
  src/biguint.rs:120-192   impl Add         -> biguint_add
  src/biguint.rs:194-265   impl Mul         -> biguint_mul (incl. the wrapping FheUint32 add into
                                               result[idx+2] at :247-249)
  src/schnorr.rs:75-141    sign / sign_with_k0 (uses privkey.value() = d' for the nonce and s even
                                               when P has odd y)
  src/schnorr.rs:235-290   sign_fhe_with_k0 (FHE block :270-277 parameterised by the limb ops)
  src/schnorr.rs:301-347   verify
  src/schnorr.rs:352-432   get_public_key_with_even_y, tagged_hash, nonce, challenge, lift_x
  src/secp256k1.rs:26-127  affine Point::new (off-curve -> infinity), add, double, scalar_mul
tfhe integer semantics used by the reference's perf_test (src/perf_test.rs:27-75): wrapping
arithmetic per width, shift amount mod width (src/biguint.rs:494-498), floor division.
"""
from __future__ import annotations

import hashlib

M32 = 1 << 32
P = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEFFFFFC2F  # src/scalar.rs:5
N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141  # src/scalar.rs:8
GX = 0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798  # src/secp256k1.rs:133
GY = 0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8


# ----------------------------------------------------------------------------- BigUintFHE
def to_u32_digits(x: int) -> list[int]:
    out = []
    while x:
        out.append(x & (M32 - 1))
        x >>= 32
    return out


def from_limbs(limbs: list[int]) -> int:
    return sum(d << (32 * i) for i, d in enumerate(limbs))


def biguint_add(a: list[int], b: list[int]) -> list[int]:
    """impl Add for BigUintFHE (src/biguint.rs:123-191), on decrypted limbs."""
    result = []
    carry = None
    for i in range(max(len(a), len(b))):
        ai = a[i] if i < len(a) else None
        bi = b[i] if i < len(b) else None
        present = [t for t in (ai, bi, carry) if t is not None]
        if carry is None and (ai is None) != (bi is None):
            result.append(ai if ai is not None else bi)  # clone arms :163-165, :175-177
            continue
        s = sum(present)  # FheUint64 adds of cast-up u32s: exact (< 2^34)
        carry = s >> 32  # cast32(sum >> 32)
        result.append(s & (M32 - 1))  # cast32(sum & 0xFFFFFFFF)
    if carry is not None:
        result.append(carry)
    return result


def biguint_mul(a: list[int], b: list[int]) -> list[int]:
    """impl Mul for BigUintFHE (src/biguint.rs:197-264), on decrypted limbs."""
    if not a or not b:
        return []
    result = [0] * (len(a) + len(b))
    for i, ai in enumerate(a):
        for j, bj in enumerate(b):
            idx = i + j
            product = ai * bj  # FheUint64 * FheUint64 (< 2^64)
            lower, upper = product & (M32 - 1), product >> 32
            s = result[idx] + lower  # FheUint64 add
            result[idx] = s & (M32 - 1)
            s = result[idx + 1] + upper + (s >> 32)
            result[idx + 1] = s & (M32 - 1)
            if idx + 2 < len(result):
                result[idx + 2] = (result[idx + 2] + (s >> 32)) % M32  # FheUint32 add: wraps
    return result


# ----------------------------------------------------------------------------- secp256k1
INF = None


def _inv(x: int, m: int) -> int:
    return pow(x, -1, m)


def on_curve(x: int, y: int) -> bool:
    return (y * y - x * x * x - 7) % P == 0


def point_new(x: int, y: int):
    """Point::new(x, y, false): off-curve coordinates become the point at infinity."""
    return (x % P, y % P) if on_curve(x, y) else INF


def point_add(p1, p2):
    if p1 is INF:
        return p2
    if p2 is INF:
        return p1
    (x1, y1), (x2, y2) = p1, p2
    if x1 == x2:
        if y1 == y2:
            lam = (3 * x1 * x1) * _inv(2 * y1, P) % P
            x3 = (lam * lam - 2 * x1) % P
            return point_new(x3, (lam * (x1 - x3) - y1) % P)
        if y1 == (-y2) % P:
            return INF
    lam = (y2 - y1) * _inv(x2 - x1, P) % P
    x3 = (lam * lam - x1 - x2) % P
    return point_new(x3, (lam * (x1 - x3) - y1) % P)


def scalar_mul(pt, k: int):
    k %= N  # Scalar::new reduces mod n (src/scalar.rs)
    result, cur = INF, pt
    while k:
        if k & 1:
            result = point_add(result, cur)
        cur = point_add(cur, cur)
        k >>= 1
    return result


G = (GX, GY)


def neg(pt):
    return INF if pt is INF else (pt[0], (-pt[1]) % P)


# ----------------------------------------------------------------------------- BIP-340
def tagged_hash(tag: bytes, msg: bytes) -> bytes:
    th = hashlib.sha256(tag).digest()
    return hashlib.sha256(th + th + msg).digest()


def b32(x: int) -> bytes:
    return x.to_bytes(32, "big")


def pubkey_even_y(d: int):
    pt = scalar_mul(G, d)
    if pt[1] % 2 == 1:
        return point_new(pt[0], P - pt[1])
    return pt


def compute_nonce(d: int, pubkey, msg: bytes, aux: bytes) -> int:
    t = bytes(x ^ y for x, y in zip(b32(d), tagged_hash(b"BIP0340/aux", aux)))
    return int.from_bytes(tagged_hash(b"BIP0340/nonce", t + b32(pubkey[0]) + msg), "big") % N


def compute_challenge(r, pubkey, msg: bytes) -> int:
    rx = 0 if r is INF else r[0]
    return int.from_bytes(tagged_hash(b"BIP0340/challenge", b32(rx) + b32(pubkey[0]) + msg), "big") % N


def sign_with_k0(msg: bytes, k0: int, d: int, mul=None, add=None):
    """Schnorr::sign_with_k0 (src/schnorr.rs:114-141); with `mul`/`add` over limb lists it is the
    FHE data flow of sign_fhe_with_k0 (src/schnorr.rs:270-276)."""
    d %= N
    pubkey = pubkey_even_y(d)
    r = scalar_mul(G, k0)
    k = (N - k0) if r[1] % 2 == 1 else k0
    e = compute_challenge(r, pubkey, msg)
    if mul is None:
        s = (k + e * d) % N
    else:
        prod = mul(to_u32_digits(e), to_u32_digits(d))
        s = from_limbs(add(to_u32_digits(k), prod)) % N
    return b32(r[0]) + b32(s)


def sign(msg: bytes, aux: bytes, d: int) -> bytes:
    """Schnorr::sign (src/schnorr.rs:75-103): nonce from d' (privkey.value())."""
    d %= N
    pubkey = pubkey_even_y(d)
    k0 = compute_nonce(d, pubkey, msg, aux)
    return sign_with_k0(msg, k0, d)


def sign_fhe_limb_flow(msg: bytes, k0: int, d: int) -> dict:
    """Intermediate values of sign_fhe_with_k0's FHE block (golden vectors)."""
    d %= N
    pubkey = pubkey_even_y(d)
    r = scalar_mul(G, k0)
    k = (N - k0) if r[1] % 2 == 1 else k0
    e = compute_challenge(r, pubkey, msg)
    e_l, d_l, k_l = to_u32_digits(e), to_u32_digits(d), to_u32_digits(k)
    prod = biguint_mul(e_l, d_l)
    ssum = biguint_add(k_l, prod)
    return {"e": e_l, "d": d_l, "k": k_l, "prod": prod, "sum": ssum,
            "s": from_limbs(ssum) % N, "r_x": r[0]}


def lift_x(x: int):
    if x >= N:  # src/schnorr.rs:423 compares against the curve order
        return INF
    y = pow((pow(x, 3, P) + 7) % P, (P + 1) // 4, P)
    if y % 2 == 1:
        y = P - y
    return point_new(x, y)


def verify(msg: bytes, pubkey_bytes: bytes, sig: bytes) -> bool:
    """Schnorr::verify (src/schnorr.rs:301-347)."""
    if len(pubkey_bytes) != 32 or len(sig) != 64:
        return False
    rx = int.from_bytes(sig[:32], "big") % P
    s = int.from_bytes(sig[32:], "big") % N
    pk = lift_x(int.from_bytes(pubkey_bytes, "big") % P)
    if pk is INF:
        return False
    ry = pow((pow(rx, 3, P) + 7) % P, (P + 1) // 4, P)
    if ry % 2 == 1:
        ry = P - ry
    r_point = point_new(rx, ry)
    r_x_of_point = 0 if r_point is INF else r_point[0]
    if r_x_of_point >= N or s >= N:
        return False
    sg = scalar_mul(G, s)
    e = compute_challenge(r_point, pk, msg)
    ep = scalar_mul(pk, e)
    rc = point_add(sg, neg(ep))
    return not (rc is INF or rc[1] % 2 == 1 or rc[0] != rx)


# ----------------------------------------------------------------------------- tfhe integer semantics
def u_add(a, b, bits):
    return (a + b) % (1 << bits)


def u_sub(a, b, bits):
    return (a - b) % (1 << bits)


def u_and(a, b, bits):
    return (a & b) % (1 << bits)


def u_mul(a, b, bits):
    return (a * b) % (1 << bits)


def u_shr(a, s, bits):
    return a >> (s % bits)


def u_shl(a, s, bits):
    return (a << (s % bits)) % (1 << bits)


def u_div(a, d):
    return a // d
