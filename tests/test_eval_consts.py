"""Constants the constraint evaluator hard-codes (csrc/kernels.hip adj_row, ZK_INV3_72) checked against
the Rescue MDS / INV_MDS tables of the reference (crypto/src/rescue.rs:197-233, generated into
csrc/rescue_consts.hpp) with Python integers: INV_MDS = adj(MDS) / 3^24, |adj| < 2^40, 3^72 * ZK_INV3_72 = 1,
and the accumulator offset p * 2^41."""
import re
from pathlib import Path

CSRC = Path(__file__).resolve().parent.parent / "encrypt-zkvm_amd" / "csrc"
P = 2**128 - 45 * 2**40 + 1


def _table(text, name):
    body = text[text.index(name):]
    body = body[:body.index("};")]
    pairs = re.findall(r"\{0x([0-9a-fA-F]+)ULL,\s*0x([0-9a-fA-F]+)ULL\}", body)
    return [int(lo, 16) | (int(hi, 16) << 64) for lo, hi in pairs]


def _signed(v):
    return v - P if v > P // 2 else v


def _kernel_text():
    return (CSRC / "kernels.hip").read_text()


def test_adjugate_is_scaled_inverse_mds():
    consts = (CSRC / "rescue_consts.hpp").read_text()
    mds = [_signed(v) for v in _table(consts, "ZK_MDS[16][2]")]
    inv = _table(consts, "ZK_INV_MDS[16][2]")
    src = _kernel_text()
    body = src[src.index("constexpr uint64_t A[16] = {"):]
    body = body[:body.index("};")]
    a = [int(x) for x in re.findall(r"(\d+)ull", body)]
    assert len(a) == 16 and max(a) < 2**40
    adj = [[a[4 * r + c] * (1 if c % 2 == 0 else -1) for c in range(4)] for r in range(4)]
    M = [[mds[4 * r + c] for c in range(4)] for r in range(4)]
    det = 3**24
    for r in range(4):
        for c in range(4):
            assert sum(adj[r][k] * M[k][c] for k in range(4)) == (det if r == c else 0)
    inv_det = pow(det, P - 2, P)
    for r in range(4):
        for c in range(4):
            assert adj[r][c] * inv_det % P == inv[4 * r + c]


def test_inverse_power_of_three_and_offset():
    src = _kernel_text()
    m = re.search(r"ZK_INV3_72 = fe\{0x([0-9a-f]+)ull, 0x([0-9a-f]+)ull\}", src)
    v = int(m.group(1), 16) | (int(m.group(2), 16) << 64)
    assert v * pow(3, 72, P) % P == 1
    m = re.search(r"uint32_t pos\[6\] = \{([^}]*)\}", src)
    words = [int(w.strip().rstrip("u"), 16) for w in m.group(1).split(",")]
    assert sum(w << (32 * i) for i, w in enumerate(words)) == P << 41
    # pos - neg stays non-negative and below 2^192: each of pos, neg gathers two 128-bit x |adj| products
    body = src[src.index("constexpr uint64_t A[16] = {"):]
    amax = max(int(x) for x in re.findall(r"(\d+)ull", body[:body.index("};")]))
    bound = 2 * 2**128 * amax
    assert (P << 41) > bound and (P << 41) + bound < 2**192
