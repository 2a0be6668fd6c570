#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/ (run in the dev
container, where /root/reference exists; the fixtures travel, the reference
does not).

Sources, in order of authority:
  * data the reference holds: the KZG trusted setup points
    (presets/mainnet/trusted_setups/trusted_setup_4096.json), the
    staking-deposit-cli Verify known answer
    (E/test/capella/block_processing/test_process_bls_to_execution_change.py:257-288),
    the altair/bls verdicts (E/test/altair/bls/*.py) and their inputs
    (E/test/altair/bls/constants.py:10-38);
  * outputs of oracle/bls_oracle.py (itself pinned by the above) for bytes
    the reference computes at generation time (signatures, aggregates,
    hash_to_G2 points) and for adversarial cases.
E = tests/core/pyspec/eth2spec of the reference.
"""
import hashlib
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle import bls_oracle as O  # noqa: E402

REF = "/root/reference"
H = lambda b: hashlib.sha256(b).digest()  # noqa: E731

# E/test/altair/bls/constants.py:10-38
MESSAGES = [b"\x00" * 32, b"\x56" * 32, b"\xab" * 32]
SAMPLE_MESSAGE = b"\x12" * 32
PRIVKEYS = [
    0x263DBD792F5B1BE47ED85F8938C0F29586AF0D3AC7B977F21C278FE1462040E3,
    0x47B8192D77BF871B62E87859D653922725724A5C031AFEABC60BCEF5FF665138,
    0x328388AFF0D4A5B7DC9205ABD374E7E98F3CD9F3418EDB4EAFDA5FB16473D216,
]
ZERO_PUBKEY = b"\x00" * 48
G1_POINT_AT_INFINITY = b"\xc0" + b"\x00" * 47
ZERO_SIGNATURE = b"\x00" * 96
G2_POINT_AT_INFINITY = b"\xc0" + b"\x00" * 95


def hx(b):
    return "0x" + bytes(b).hex()


def dump(name, obj):
    with open(os.path.join(HERE, name), "w") as fh:
        json.dump(obj, fh, indent=1)
    print("wrote", name)


def altair_bls():
    """The 20 runner=bls cases, in tests/formats/bls layout."""
    cases = []
    # test_eth_aggregate_pubkeys.py:14-108
    for i, sk in enumerate(PRIVKEYS):
        pk = O.SkToPk(sk)
        cases.append({"handler": "eth_aggregate_pubkeys", "case": f"eth_aggregate_pubkeys_valid_{i}",
                      "input": [hx(pk)], "output": hx(O.AggregatePKs([pk]))})
    pks = [O.SkToPk(sk) for sk in PRIVKEYS]
    cases.append({"handler": "eth_aggregate_pubkeys", "case": "eth_aggregate_pubkeys_valid_pubkeys",
                  "input": [hx(p) for p in pks], "output": hx(O.AggregatePKs(pks))})
    for name, inp in (("empty_list", []), ("zero_pubkey", [ZERO_PUBKEY]), ("infinity_pubkey", [G1_POINT_AT_INFINITY]),
                      ("x40_pubkey", [b"\x40" + b"\x00" * 47])):
        cases.append({"handler": "eth_aggregate_pubkeys", "case": f"eth_aggregate_pubkeys_{name}",
                      "input": [hx(p) for p in inp], "output": None})  # None == must raise
    # test_eth_fast_aggregate_verify.py:19-151
    for mi, msg in enumerate(MESSAGES):
        sks = PRIVKEYS[: mi + 1]
        agg = O.Aggregate([O.Sign(sk, msg) for sk in sks])
        pk = [O.SkToPk(sk) for sk in sks]
        cases.append({"handler": "eth_fast_aggregate_verify", "case": f"eth_fast_aggregate_verify_valid_{mi}",
                      "input": {"pubkeys": [hx(p) for p in pk], "message": hx(msg), "signature": hx(agg)},
                      "output": True})
        cases.append({"handler": "eth_fast_aggregate_verify", "case": f"eth_fast_aggregate_verify_extra_pubkey_{mi}",
                      "input": {"pubkeys": [hx(p) for p in pk + [O.SkToPk(PRIVKEYS[-1])]], "message": hx(msg),
                                "signature": hx(agg)}, "output": False})
        tampered = agg[:-4] + b"\xff\xff\xff\xff"
        cases.append({"handler": "eth_fast_aggregate_verify",
                      "case": f"eth_fast_aggregate_verify_tampered_signature_{mi}",
                      "input": {"pubkeys": [hx(p) for p in pk], "message": hx(msg), "signature": hx(tampered)},
                      "output": False})
    cases.append({"handler": "eth_fast_aggregate_verify", "case": "eth_fast_aggregate_verify_na_pubkeys_and_infinity_signature",
                  "input": {"pubkeys": [], "message": hx(MESSAGES[-1]), "signature": hx(G2_POINT_AT_INFINITY)},
                  "output": True})
    cases.append({"handler": "eth_fast_aggregate_verify", "case": "eth_fast_aggregate_verify_na_pubkeys_and_zero_signature",
                  "input": {"pubkeys": [], "message": hx(MESSAGES[-1]), "signature": hx(ZERO_SIGNATURE)},
                  "output": False})
    agg = O.Aggregate([O.Sign(sk, SAMPLE_MESSAGE) for sk in PRIVKEYS])
    cases.append({"handler": "eth_fast_aggregate_verify", "case": "eth_fast_aggregate_verify_infinity_pubkey",
                  "input": {"pubkeys": [hx(O.SkToPk(sk)) for sk in PRIVKEYS] + [hx(G1_POINT_AT_INFINITY)],
                            "message": hx(SAMPLE_MESSAGE), "signature": hx(agg)},
                  "output": False})
    # cross-check the oracle against the hard-coded verdicts of the reference tests
    for c in cases:
        if c["handler"] == "eth_fast_aggregate_verify":
            i = c["input"]
            got = O.eth_fast_aggregate_verify([bytes.fromhex(p[2:]) for p in i["pubkeys"]],
                                              bytes.fromhex(i["message"][2:]), bytes.fromhex(i["signature"][2:]))
            assert got == c["output"], c["case"]
    assert len(cases) == 20
    return cases


def bls_formats():
    """verify / aggregate / fast_aggregate_verify / aggregate_verify / sign handlers
    (tests/formats/bls/*.md layouts), generated by the oracle, incl. edge cases."""
    out = {"sign": [], "verify": [], "aggregate": [], "fast_aggregate_verify": [], "aggregate_verify": [],
           "sk_to_pk": [], "key_validate": []}
    for sk in PRIVKEYS:
        out["sk_to_pk"].append({"input": hx(sk.to_bytes(32, "big")), "output": hx(O.SkToPk(sk))})
        for m in MESSAGES:
            out["sign"].append({"input": {"privkey": hx(sk.to_bytes(32, "big")), "message": hx(m)},
                                "output": hx(O.Sign(sk, m))})
    out["sign"].append({"input": {"privkey": hx(bytes(32)), "message": hx(MESSAGES[0])}, "output": None})
    out["sign"].append({"input": {"privkey": hx(O.R.to_bytes(32, "big")), "message": hx(MESSAGES[0])}, "output": None})
    pk0, sig00 = O.SkToPk(PRIVKEYS[0]), O.Sign(PRIVKEYS[0], MESSAGES[0])
    vcases = [
        (pk0, MESSAGES[0], sig00, True),
        (pk0, MESSAGES[1], sig00, False),                      # wrong message
        (O.SkToPk(PRIVKEYS[1]), MESSAGES[0], sig00, False),    # wrong pubkey
        (pk0, MESSAGES[0], sig00[:-4] + b"\xff" * 4, False),   # tampered
        (pk0, MESSAGES[0], G2_POINT_AT_INFINITY, False),       # infinity signature
        (pk0, MESSAGES[0], ZERO_SIGNATURE, False),             # not a valid encoding
        (G1_POINT_AT_INFINITY, MESSAGES[0], G2_POINT_AT_INFINITY, False),  # infinity pubkey
        (ZERO_PUBKEY, MESSAGES[0], sig00, False),
        (pk0, b"", O.Sign(PRIVKEYS[0], b""), True),            # empty message
        (pk0, b"x" * 100, O.Sign(PRIVKEYS[0], b"x" * 100), True),  # long message
    ]
    for pk, m, s, exp in vcases:
        assert O.Verify(pk, m, s) == exp
        out["verify"].append({"input": {"pubkey": hx(pk), "message": hx(m), "signature": hx(s)}, "output": exp})
    for m in MESSAGES:
        sigs = [O.Sign(sk, m) for sk in PRIVKEYS]
        out["aggregate"].append({"input": [hx(s) for s in sigs], "output": hx(O.Aggregate(sigs))})
    out["aggregate"].append({"input": [hx(sig00)], "output": hx(sig00)})
    out["aggregate"].append({"input": [hx(G2_POINT_AT_INFINITY)], "output": hx(G2_POINT_AT_INFINITY)})
    out["aggregate"].append({"input": [hx(sig00), hx(O.g2_compress(O.g2_neg(O.g2_decompress(sig00))))],
                             "output": hx(G2_POINT_AT_INFINITY)})
    out["aggregate"].append({"input": [], "output": None})
    out["aggregate"].append({"input": [hx(ZERO_SIGNATURE)], "output": None})
    nonsub = O.g2_compress(O.iso_map(O.map_to_curve_sswu((3, 4))))
    out["aggregate"].append({"input": [hx(nonsub)], "output": None})
    # FAV / AV
    pks = [O.SkToPk(sk) for sk in PRIVKEYS]
    for m in MESSAGES:
        agg = O.Aggregate([O.Sign(sk, m) for sk in PRIVKEYS])
        out["fast_aggregate_verify"].append({"input": {"pubkeys": [hx(p) for p in pks], "message": hx(m),
                                                       "signature": hx(agg)}, "output": True})
        out["fast_aggregate_verify"].append({"input": {"pubkeys": [hx(p) for p in pks[:2]], "message": hx(m),
                                                       "signature": hx(agg)}, "output": False})
    out["fast_aggregate_verify"].append({"input": {"pubkeys": [], "message": hx(MESSAGES[0]),
                                                   "signature": hx(G2_POINT_AT_INFINITY)}, "output": False})
    negpk = O.g1_compress(O.g1_neg(O.g1_decompress(pks[0])))
    out["fast_aggregate_verify"].append({"input": {"pubkeys": [hx(pks[0]), hx(negpk)], "message": hx(MESSAGES[0]),
                                                   "signature": hx(G2_POINT_AT_INFINITY)}, "output": False})
    sigs = [O.Sign(sk, m) for sk, m in zip(PRIVKEYS, MESSAGES)]
    agg = O.Aggregate(sigs)
    out["aggregate_verify"].append({"input": {"pubkeys": [hx(p) for p in pks], "messages": [hx(m) for m in MESSAGES],
                                              "signature": hx(agg)}, "output": True})
    out["aggregate_verify"].append({"input": {"pubkeys": [hx(p) for p in pks], "messages": [hx(m) for m in MESSAGES[::-1]],
                                              "signature": hx(agg)}, "output": False})
    out["aggregate_verify"].append({"input": {"pubkeys": [hx(p) for p in pks[:2]], "messages": [hx(m) for m in MESSAGES],
                                              "signature": hx(agg)}, "output": False})
    out["aggregate_verify"].append({"input": {"pubkeys": [], "messages": [], "signature": hx(G2_POINT_AT_INFINITY)},
                                    "output": False})
    out["aggregate_verify"].append({"input": {"pubkeys": [hx(p) for p in pks], "messages": [hx(m) for m in MESSAGES],
                                              "signature": hx(agg[:-4] + b"\xff" * 4)}, "output": False})
    for c in out["aggregate_verify"]:
        i = c["input"]
        assert O.AggregateVerify([bytes.fromhex(p[2:]) for p in i["pubkeys"]], [bytes.fromhex(m[2:]) for m in i["messages"]],
                                 bytes.fromhex(i["signature"][2:])) == c["output"]
    # KeyValidate edges (E/test/phase0/block_processing/test_process_deposit.py:255-287)
    x = 1
    while True:
        y = O.fp_sqrt(x ** 3 + 4)
        if y is not None and not O.g1_in_subgroup((x, y)):
            break
        x += 1
    for enc, exp in ((pk0, True), (ZERO_PUBKEY, False), (G1_POINT_AT_INFINITY, False),
                     (bytes([0xC0, 0x10]) + bytes(46), False), (b"\x40" + bytes(47), False),
                     (O.g1_compress((x, y)), False), ((O.P | (1 << 383)).to_bytes(48, "big"), False),
                     (negpk, True)):
        assert O.KeyValidate(enc) == exp
        out["key_validate"].append({"input": hx(enc), "output": exp})
    return out


def hash_to_g2_vectors():
    rng = random.Random(0x5EED)
    msgs = [b"", b"abc", bytes(32), b"\x56" * 32, b"\xab" * 32] + [bytes(rng.randrange(256) for _ in range(32)) for _ in range(5)]
    res = []
    for m in msgs:
        res.append({"msg": hx(m), "dst": O.DST_POP.decode(), "output": hx(O.g2_compress(O.hash_to_g2(m)))})
    qd = b"QUUX-V01-CS02-with-BLS12381G2_XMD:SHA-256_SSWU_RO_"
    for m in (b"", b"abc"):
        res.append({"msg": hx(m), "dst": qd.decode(), "output": hx(O.g2_compress(O.hash_to_g2(m, qd)))})
    return res


def known_answers():
    pk = bytes.fromhex("86248e64705987236ec3c41f6a81d96f98e7b85e842a1d71405b216fa75a9917512f3c94c85779a9729c927ea2aa9ed1")
    sig = bytes.fromhex("8cf4219884b326a04f6664b680cd9a99ad70b5280745af1147477aa9f8b4a2b2b38b8688c6a74a06f275ad4e14c5c0c7"
                        "0e2ed37a15ece5bf7c0724a376ad4c03c79e14dd9f633a3d54abc1ce4e73bec3524a789ab9a69d4d06686a8a67c9e4dc")
    gvr = bytes.fromhex("4b363db94e286120d76eb905340fdd4e54bfe9f06bf33ff6cf5ad27f511bfe95")
    # SSZ hash_tree_root(BLSToExecutionChange{validator_index=1, from_bls_pubkey=pk, to_execution_address=0x34*20})
    c0 = (1).to_bytes(8, "little") + bytes(24)
    c1 = H(pk[:32] + pk[32:] + bytes(16))
    c2 = b"\x34" * 20 + bytes(12)
    root = H(H(c0 + c1) + H(c2 + bytes(32)))
    domain = bytes.fromhex("0a000000") + H(bytes(32) + gvr)[:28]  # compute_domain(DOMAIN_BLS_TO_EXECUTION_CHANGE)
    sr = H(root + domain)
    assert sr.hex() == "ea9b5656a364bc4d92aca5806b91a76fe538217e39e258d1b9874e776cb49904"
    assert O.Verify(pk, sr, sig)
    return {"deposit_cli": {"pubkey": hx(pk), "signing_root": hx(sr), "signature": hx(sig), "output": True},
            "deposit_cli_flipped": {"pubkey": hx(pk), "signing_root": hx(bytes([sr[0] ^ 1]) + sr[1:]),
                                    "signature": hx(sig), "output": False}}


def trusted_setup():
    d = json.load(open(os.path.join(REF, "presets/mainnet/trusted_setups/trusted_setup_4096.json")))
    return {"source": "presets/mainnet/trusted_setups/trusted_setup_4096.json",
            "g1_lagrange": d["g1_lagrange"], "g1_monomial": d["g1_monomial"][:66], "g2_monomial": d["g2_monomial"]}


if __name__ == "__main__":
    dump("altair_bls.json", altair_bls())
    dump("bls_formats.json", bls_formats())
    dump("hash_to_g2.json", hash_to_g2_vectors())
    dump("known_answers.json", known_answers())
    dump("trusted_setup.json", trusted_setup())
