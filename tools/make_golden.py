#!/usr/bin/env python3
"""Generate tests/golden/*.json from the plaintext restatement (oracle/ref_semantics.py) and the
reference's own known answers.  Committed together with the fixtures it writes.

Sources:
  known answers transcribed from the reference tests:
    src/biguint.rs:274-526, src/schnorr.rs:575-607, src/perf_test.rs:14-75
  tests/golden/bip340_vectors.csv = the reference's tests/test_vectors.csv (data file, verbatim)
  generated vectors: random 256-bit limbs (seed 0xF11E51), quirk inputs (F7),
  and the sign_fhe_with_k0 limb flow for every BIP-340 signing vector.
"""
import csv
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import ref_semantics as R  # noqa: E402

G = os.path.join(ROOT, "tests", "golden")

known = {
    "source": "reference unit tests (src/biguint.rs, src/schnorr.rs, src/perf_test.rs)",
    "biguint": [
        {"test": "test_mul_with_carry_small_numbers src/biguint.rs:274", "op": "mul", "a": 2, "b": 3, "value": 6},
        {"test": "test_biguint_conversion src/biguint.rs:295", "op": "roundtrip", "a": 123456789123456789, "value": 123456789123456789},
        {"test": "test_add_with_carry src/biguint.rs:308", "op": "add", "a": 0xFFFFFFFF, "b": 1, "limbs": [0, 1]},
        {"test": "test_mul_with_carry src/biguint.rs:336", "op": "mul", "a": 0xFFFFFFFF, "b": 2, "limbs": [0xFFFFFFFE, 1]},
        {"test": "test_mul_with_carry_2 src/biguint.rs:354", "op": "mul", "a": 0xFFFFFFFF, "b": 0xFFFFFFFF, "limbs": [1, 0xFFFFFFFE]},
        {"test": "test_add_multiple_carries src/biguint.rs:372", "op": "add", "a": 0xFFFFFFFF, "b": 0xFFFFFFFF, "limbs": [0xFFFFFFFE, 1]},
        {"test": "test_mul_multiple_carries src/biguint.rs:389", "op": "mul", "a": 0xFFFFFFFF, "b": 0xFFFFFFFF, "limbs": [1, 0xFFFFFFFE]},
        {"test": "test_large_number_operations src/biguint.rs:407 (add)", "op": "add", "a": 123456789123456789, "b": 987654321987654321,
         "value": 123456789123456789 + 987654321987654321},
        {"test": "test_large_number_operations src/biguint.rs:407 (mul)", "op": "mul", "a": 123456789123456789, "b": 987654321987654321,
         "value": 123456789123456789 * 987654321987654321},
    ],
    "fheuint": [
        {"test": "test_extract_carry_and_lower_bits src/biguint.rs:429 #1", "bits": 64, "a": 5, "b": 3, "op": "add_split", "hi": 0, "lo": 8},
        {"test": "test_extract_carry_and_lower_bits src/biguint.rs:429 #2", "bits": 64, "a": 0xFFFFFFFF, "b": 1, "op": "add_split", "hi": 1, "lo": 0},
        {"test": "test_extract_carry_and_lower_bits src/biguint.rs:429 #3", "bits": 64, "a": 0xFFFFFFFF, "b": 0xFFFFFFFF, "op": "add_split", "hi": 1, "lo": 0xFFFFFFFE},
        {"test": "test_uint64_carry_behavior src/biguint.rs:502", "bits": 64, "a": 0xFFFFFFFF, "b": 1, "op": "add_shr_and", "hi": 1, "lo": 0},
        {"test": "test_uint32_overflow_behavior src/biguint.rs:469 (documented in comments :494-498)", "bits": 32, "a": 0xFFFFFFFF, "b": 1,
         "op": "add_shr_and", "hi": 0, "lo": 0},
        {"test": "test_uint32_overflow_behavior src/biguint.rs:469 (second case)", "bits": 32, "a": 0xFFFFFFFF, "b": 0xFFFFFFFF,
         "op": "add_shr_and", "hi": 0xFFFFFFFE, "lo": 0xFFFFFFFE},
        {"test": "test_fheu32_mul_u32 src/schnorr.rs:575", "bits": 32, "a": 123, "b": 456, "op": "scalar_mul", "value": 56088},
        {"test": "test_fheu32_add_u32 src/schnorr.rs:595", "bits": 32, "a": 123, "b": 456, "op": "scalar_add", "value": 579},
        {"test": "perf_test src/perf_test.rs:28", "bits": 32, "a": 1344, "b": 5, "op": "add", "value": 1349},
        {"test": "perf_test src/perf_test.rs:32", "bits": 32, "a": 1344, "b": 5, "op": "mul", "value": 6720},
        {"test": "perf_test src/perf_test.rs:36-63", "bits": 32, "a": 1344, "b": 5, "c": 7, "op": "perf_chain", "value": 1},
        {"test": "perf_test src/perf_test.rs:54,75", "bits": 32, "a": 1344, "b": 5, "op": "scalar_div", "value": 268},
    ],
}

rng = random.Random(0xF11E51)


def r256():
    return rng.getrandbits(256) | (1 << 255)


gen = {"source": "oracle/ref_semantics.py (restatement of src/biguint.rs:120-265), seed 0xF11E51",
       "add": [], "mul": [], "quirk_mul": []}
for _ in range(32):
    a, b = r256(), r256()
    A, B = R.to_u32_digits(a), R.to_u32_digits(b)
    gen["add"].append({"a": A, "b": B, "out": R.biguint_add(A, B)})
for _ in range(8):
    a, b = r256(), r256()
    A, B = R.to_u32_digits(a), R.to_u32_digits(b)
    gen["mul"].append({"a": A, "b": B, "out": R.biguint_mul(A, B)})
# carry-loss quirk: results differ from the true product
ones = (1 << 256) - 1
for a, b in ((ones, ones), ((1 << 96) - 1, (1 << 96) - 1), (ones, (1 << 64) - 1)):
    A, B = R.to_u32_digits(a), R.to_u32_digits(b)
    out = R.biguint_mul(A, B)
    gen["quirk_mul"].append({"a": A, "b": B, "out": out, "true_product": R.to_u32_digits(a * b),
                             "differs": R.from_limbs(out) != a * b})
gen["edge"] = [
    {"op": "add", "a": [], "b": [5, 6], "out": R.biguint_add([], [5, 6])},
    {"op": "add", "a": [1, 2, 3], "b": [], "out": R.biguint_add([1, 2, 3], [])},
    {"op": "mul", "a": [], "b": [5], "out": R.biguint_mul([], [5])},
    {"op": "add", "a": [7], "b": [1, 2, 3], "out": R.biguint_add([7], [1, 2, 3])},
    {"op": "mul", "a": [0xFFFFFFFF] * 3, "b": [0xFFFFFFFF], "out": R.biguint_mul([0xFFFFFFFF] * 3, [0xFFFFFFFF])},
]

sign = {"source": "tests/golden/bip340_vectors.csv + oracle/ref_semantics.py", "vectors": []}
with open(os.path.join(G, "bip340_vectors.csv")) as f:
    for row in csv.DictReader(f):
        if not row["secret key"]:
            continue
        d = int(row["secret key"], 16)
        msg, aux = bytes.fromhex(row["message"]), bytes.fromhex(row["aux_rand"])
        pk = R.pubkey_even_y(d % R.N)
        k0 = R.compute_nonce(d % R.N, pk, msg, aux)
        flow = R.sign_fhe_limb_flow(msg, k0, d)
        sig = R.sign_with_k0(msg, k0, d)
        sign["vectors"].append({
            "index": int(row["index"]), "seckey": row["secret key"], "message": row["message"], "k0": hex(k0),
            "csv_signature": row["signature"], "sign_with_k0": sig.hex().upper(),
            "matches_csv": sig.hex().upper() == row["signature"].upper(), **{k: (v if not isinstance(v, int) else hex(v)) for k, v in flow.items()}})

for name, obj in (("known_answers.json", known), ("biguint_vectors.json", gen), ("sign_vectors.json", sign)):
    with open(os.path.join(G, name), "w") as f:
        json.dump(obj, f, indent=1)
print("wrote", os.listdir(G))
