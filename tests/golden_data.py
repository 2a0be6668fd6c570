"""Known answers taken from the reference's own tests (not generated here).

DEPOSIT_CLI: E/test/capella/block_processing/test_process_bls_to_execution_change.py:257-288
(a real staking-deposit-cli signature verified with mainnet parameters).  The
signing root is the SSZ root of BLSToExecutionChange{1, pk, 0x34*20} under
DOMAIN_BLS_TO_EXECUTION_CHANGE with GENESIS_FORK_VERSION 0x00000000 and the
mainnet genesis_validators_root; tests/golden/make_golden.py recomputes it
with hashlib only.
"""
DEPOSIT_CLI = {
    "pubkey": bytes.fromhex(
        "86248e64705987236ec3c41f6a81d96f98e7b85e842a1d71405b216fa75a9917512f3c94c85779a9729c927ea2aa9ed1"),
    "signature": bytes.fromhex(
        "8cf4219884b326a04f6664b680cd9a99ad70b5280745af1147477aa9f8b4a2b2b38b8688c6a74a06f275ad4e14c5c0c7"
        "0e2ed37a15ece5bf7c0724a376ad4c03c79e14dd9f633a3d54abc1ce4e73bec3524a789ab9a69d4d06686a8a67c9e4dc"),
    "signing_root": bytes.fromhex("ea9b5656a364bc4d92aca5806b91a76fe538217e39e258d1b9874e776cb49904"),
    "genesis_validators_root": bytes.fromhex("4b363db94e286120d76eb905340fdd4e54bfe9f06bf33ff6cf5ad27f511bfe95"),
}
