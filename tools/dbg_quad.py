import os, sys, numpy as np
sys.path.insert(0, 'fhe-sign_amd'); sys.path.insert(0, 'oracle')
import oracle
from fhe_sign import Context, generate_keys
ck, sk = generate_keys(seed=0xC0FFEE)
ok = oracle.OracleKeys(0xC0FFEE)
ctx = Context(0); ctx.set_server_key(sk)
lid = ctx.lut([(m + 1) % 16 for m in range(16)])
NB = int(sys.argv[1]); r = ok.rng(5)
cts = np.stack([ok.encrypt(r, i % 16) for i in range(NB)])
ctx.set_wide_threshold(1 << 30); wide = ctx.pbs(cts, lid)
ctx.set_wide_threshold(0); quad = ctx.pbs(cts, lid)
bad = [i for i in range(NB) if not np.array_equal(wide[i], quad[i])]
print("bad cts", len(bad), bad[:10])
if bad:
    i = bad[0]; d = np.flatnonzero(wide[i] != quad[i]); print("words differ", d.size, d[:10], d[-5:])
    print("decrypt wide", ok.decrypt(wide[i]), "quad", ok.decrypt(quad[i]))
