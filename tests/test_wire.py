"""Wire formats (zkvm_amd.wire): vint64 usize, Hash serde, the proof walker and OutputData, on the
golden proofs (CPU; the verifier is the library's zk_verify)."""
import json
from pathlib import Path

import pytest

from zkvm_amd import wire
from zkvm_amd.prover import make_pub_inputs, verify

GOLD = Path(__file__).resolve().parent / "golden"
CASES = json.loads((GOLD / "cases.json").read_text())["cases"]


def ints(hs):
    return [int(h, 16) for h in hs]


@pytest.mark.parametrize("v,enc", [(0, b"\x01"), (16, b"\x21"), (127, b"\xff"), (128, b"\x02\x02"),
                                   (2**64 - 1, b"\x00" + b"\xff" * 8)])
def test_usize_vint64(v, enc):
    assert wire.write_usize(v) == enc
    assert wire.read_usize(enc, 0) == (v, len(enc))


def test_usize_roundtrip_all_lengths():
    for bits in range(0, 64):
        for v in (1 << bits, (1 << bits) - 1, (1 << bits) + 12345 % (1 << max(bits, 1))):
            if v < 2**64:
                e = wire.write_usize(v)
                assert wire.read_usize(e + b"tail", 0) == (v, len(e))


@pytest.mark.parametrize("c", CASES, ids=[c["name"] for c in CASES])
def test_output_data_roundtrip(c):
    proof = (GOLD / f"{c['name']}.proof").read_bytes()
    view, end = wire.parse_proof(proof)
    assert end == len(proof) and view.raw == proof
    o = c["options"]
    assert (view.num_queries, view.blowup, view.grinding, view.field_extension, view.fri_folding,
            view.fri_rem_max_deg) == (o["num_queries"], o["blowup"], o["grinding"], o["field_extension"],
                                      o["fri_folding"], o["fri_rem_max_deg"])
    assert view.pow_nonce == c["pow_nonce"]
    h, outs = ints(c["program_hash"]), ints(c["stack_outputs"])
    blob = wire.OutputData(h, proof, outs).to_bytes()
    back = wire.OutputData.from_bytes(blob)
    assert back.hash == h and back.output == outs and back.proof == proof
    pub = make_pub_inputs(back.hash, back.output, c["lwe_size"], c["delta"])
    assert verify(back.proof, pub, 0) == (0, "")
    with pytest.raises(ValueError):
        wire.OutputData.from_bytes(blob[:-1])
    with pytest.raises(ValueError):
        wire.OutputData.from_bytes(blob + b"\x00")


def _case(name):
    c = next(c for c in CASES if c["name"] == name)
    pub = make_pub_inputs(ints(c["program_hash"]), ints(c["stack_outputs"]), c["lwe_size"], c["delta"])
    return c, (GOLD / f"{name}.proof").read_bytes(), pub


@pytest.mark.parametrize("lwe_size", [0, 6, 255])
def test_verify_rejects_lwe_size_out_of_range(lwe_size):
    """zk_verify bounds lwe_size like the prover (air_eval indexes the OOD frame with it)."""
    from zkvm_amd import native
    c, proof, pub = _case("lr")
    pub.lwe_size = lwe_size
    rc, msg = verify(proof, pub, 0)
    assert rc == native.ZK_ERR_INVALID_ARG and "lwe_size" in msg


@pytest.mark.parametrize("name", ["lr", "lr_quad"])
@pytest.mark.parametrize("delta_cols", [-1, +1])
def test_verify_requires_air_composition_width(name, delta_cols):
    """The OOD constraint frame must hold exactly num_comp_cols(n) values (winter-air derives the count
    from the AIR); a frame one column shorter or longer is malformed, not re-interpreted."""
    from zkvm_amd import native
    c, proof, pub = _case(name)
    view, _ = wire.parse_proof(proof)
    at, width, ln = view.sections["ood_evaluations"]
    es = 16 * view.field_extension
    assert width == 2 and ln % es == 0 and ln // es == 7
    body = proof[at + 2:at + 2 + ln]
    body = body[:-es] if delta_cols < 0 else body + body[:es]
    bad = proof[:at] + len(body).to_bytes(2, "little") + body + proof[at + 2 + ln:]
    rc, msg = verify(bad, pub, 0)
    assert rc == native.ZK_ERR_VERIFY and msg == "malformed out-of-domain frame"
    assert verify(proof, pub, 0) == (0, "")
