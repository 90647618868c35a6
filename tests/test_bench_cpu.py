"""bench.py host helpers (no GPU): the pin lookup behind the bench's self-checks (`proof_matches_pin` of the replica
line and of the sharded sub-record) and the exchange record of the sharded leg."""
import hashlib
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402
from zkvm_amd.prover import ProofOptions  # noqa: E402


def test_replica_workload_is_the_configs2_pin():
    pin = bench.find_pin(20, 1000, ProofOptions())
    assert pin is not None and pin["name"] == "c2_cipher_2p20"
    proof = (ROOT / "tests" / "golden" / "large" / "c2_cipher_2p20.proof").read_bytes()
    assert bench.pin_check(proof, pin) == {"pin": "c2_cipher_2p20", "proof_matches_pin": True}
    bad = bytearray(proof)
    bad[-1] ^= 1
    assert bench.pin_check(bytes(bad), pin)["proof_matches_pin"] is False
    assert bench.pin_check(proof[:-1], pin)["proof_matches_pin"] is False


def test_config5_and_sharded_pins():
    assert bench.find_pin(20, 1000, ProofOptions(43, 8, 0, 2, 8, 127))["name"] == "c4_cipher_2p20_quad"
    c3 = bench.find_pin(22, 1000, ProofOptions())
    assert c3["name"] == "c3_cipher_2p22"
    proof = (ROOT / "tests" / "golden" / "large" / "c3_cipher_2p22.proof").read_bytes()
    assert hashlib.sha256(proof).hexdigest() == c3["proof_sha256"]


def test_no_pin_for_other_ranks_or_options():
    assert bench.find_pin(20, 1001, ProofOptions()) is None  # rank 1's replica seed
    assert bench.find_pin(20, 1000, ProofOptions(num_queries=31)) is None
    assert bench.find_pin(19, 1000, ProofOptions()) is None
    assert bench.pin_check(b"x", None) is None


def test_exchange_record():
    rec = bench.exchange_record({"trace_digests": (2.0, 4e8, 1), "trace_roots": (0.01, 224.0, 1)})
    assert rec["trace_digests"] == {"ms": 2.0, "mb_received": 400.0, "calls": 1, "gb_per_s": 200.0}
    assert rec["total"]["mb_received"] == round((4e8 + 224) / 1e6, 3)
    assert bench.exchange_record({})["total"]["gb_per_s"] is None
    # with the exposed time (zk_prover_exchange_stats_ex): per collective and summed
    rec = bench.exchange_record({"a": (2.0, 4e8, 4, 0.5), "b": (1.0, 1e8, 1, 0.25)})
    assert rec["a"]["exposed_ms"] == 0.5 and rec["total"]["exposed_ms"] == 0.75


def test_model_record_reads_the_committed_projection():
    rec = bench.model_record(22, 8, False, {"device": 22.0, "host": 11.0})
    assert rec["source"] == bench.SHARD_MODEL
    assert 5.0 < rec["device"]["modelled_per_rank_ms"] < 20.0
    assert rec["device"]["measured_over_modelled"] == round(22.0 / rec["device"]["modelled_per_rank_ms"], 3)
    assert bench.model_record(20, 8, False, {"device": 1.0}) is None  # other trace length: no projection
    assert bench.model_record(22, 8, True, {"device": 1.0}) is None   # configs[4]: not modelled


def test_all_ranks_true_single_process():
    assert bench.all_ranks_true(None, True, 0) is True
    assert bench.all_ranks_true(None, False, 0) is False
