"""Wire formats around the proof bytes.

  * ``Proof::to_bytes`` / ``Proof::read_from`` (winterfell 0.9, the layout the library writes,
    DESIGN.md "Protocol profile" P13/P14): ``parse_proof`` walks it and returns the sections, so a
    proof can be found inside a larger stream.
  * ``OutputData`` (examples/linear_regression/src/utils.rs:62-128): Hash || Proof || usize(16) ||
    16 output elements, as the example writes to disk and reads back before verifying.
  * ``Hash`` serde (crypto/src/rescue.rs:87-101): two base elements, 16 B LE each.
  * ``write_usize`` / ``read_usize``: winter-utils' vint64 encoding (the length is one plus the number
    of trailing zero bits of the first byte; 9 bytes with a zero first byte above 2^56).
Parity at this layer is unpinned like the rest of the winterfell layout.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field

P = 2**128 - 45 * 2**40 + 1


def write_usize(value: int) -> bytes:
    if value < 0 or value >= 1 << 64:
        raise ValueError("usize out of range")
    zeros = 64 - value.bit_length()
    length = 9 - min(max(zeros - 1, 0) // 7, 8)
    if length == 9:
        return b"\x00" + value.to_bytes(8, "little")
    return ((((value << 1) | 1) << (length - 1)) & ((1 << (8 * length)) - 1)).to_bytes(length, "little")


def read_usize(buf: bytes, off: int) -> tuple[int, int]:
    if off >= len(buf):
        raise ValueError("truncated usize")
    first = buf[off]
    if first == 0:
        if off + 9 > len(buf):
            raise ValueError("truncated usize")
        return int.from_bytes(buf[off + 1:off + 9], "little"), off + 9
    length = (first & -first).bit_length()  # trailing zeros + 1
    if off + length > len(buf):
        raise ValueError("truncated usize")
    v = int.from_bytes(buf[off:off + length], "little") >> length
    return v, off + length


def elem_to_bytes(v: int) -> bytes:
    if not 0 <= v < P:
        raise ValueError("not a canonical f128 element")
    return v.to_bytes(16, "little")


def elem_from_bytes(b: bytes) -> int:
    v = int.from_bytes(b[:16], "little")
    if v >= P:
        raise ValueError("non-canonical f128 element")
    return v


@dataclass
class ProofView:
    """The sections of one serialized proof (byte ranges into ``raw``)."""
    raw: bytes
    trace_width: int
    trace_len: int
    num_queries: int
    blowup: int
    grinding: int
    field_extension: int
    fri_folding: int
    fri_rem_max_deg: int
    num_unique_queries: int
    commitments: bytes
    num_fri_layers: int
    pow_nonce: int
    # length-prefixed sections: name -> (offset of the length prefix in ``raw``, prefix bytes, body length)
    sections: dict = field(default_factory=dict)


class _R:
    def __init__(self, b: bytes, off: int):
        self.b, self.o = b, off

    def take(self, n: int) -> bytes:
        if self.o + n > len(self.b):
            raise ValueError("truncated proof")
        s = self.b[self.o:self.o + n]
        self.o += n
        return s

    def u8(self):
        return self.take(1)[0]

    def u16(self):
        return struct.unpack("<H", self.take(2))[0]

    def u32(self):
        return struct.unpack("<I", self.take(4))[0]

    def u64(self):
        return struct.unpack("<Q", self.take(8))[0]


def parse_proof(buf: bytes, off: int = 0) -> tuple[ProofView, int]:
    """Walk one proof starting at ``off``; returns its view and the offset just past it."""
    r = _R(buf, off)
    width, aux_w, aux_r, log_n = r.u8(), r.u8(), r.u8(), r.u8()
    r.take(r.u16())  # trace metadata
    r.take(r.u8())  # field modulus bytes
    nq, blowup, grind, ext, fold, remdeg = r.u8(), r.u8(), r.u8(), r.u8(), r.u8(), r.u8()
    nu = r.u8()
    coms = r.take(r.u16())
    for _ in range(r.u8()):  # trace segments: values + batch proof
        r.take(r.u32())
        r.take(r.u32())
    sections = {}

    def sect(name, width):
        at = r.o - off
        ln = r.u16() if width == 2 else r.u32()
        r.take(ln)
        sections[name] = (at, width, ln)

    sect("constraint_values", 4)
    sect("constraint_proof", 4)
    sect("ood_trace_states", 2)
    sect("ood_evaluations", 2)
    nl = r.u8()
    for _ in range(nl):
        r.take(r.u32())
        r.take(r.u32())
    r.take(r.u16())  # remainder
    r.u8()  # num_partitions
    nonce = r.u64()
    if r.u8():  # gkr proof: Some(..) is not produced by this AIR
        raise ValueError("unexpected GKR proof")
    view = ProofView(bytes(buf[off:r.o]), width, 1 << log_n, nq, blowup, grind, ext, fold, remdeg, nu, coms, nl, nonce,
                     sections)
    if aux_w or aux_r:
        raise ValueError("unexpected auxiliary trace segment")
    return view, r.o


def hash_to_bytes(h) -> bytes:
    """Hash::write_into: the two digest elements (crypto/src/rescue.rs:87-92)."""
    return b"".join(elem_to_bytes(v) for v in h)


def hash_from_bytes(b: bytes, off: int = 0) -> tuple[list[int], int]:
    return [elem_from_bytes(b[off:off + 16]), elem_from_bytes(b[off + 16:off + 32])], off + 32


@dataclass
class OutputData:
    """examples/linear_regression/src/utils.rs:62-128: what the example stores after proving."""
    hash: list
    proof: bytes
    output: list

    def to_bytes(self) -> bytes:
        if len(self.output) != 16:
            raise ValueError("expected 16 output elements")
        return (hash_to_bytes(self.hash) + self.proof + write_usize(len(self.output)) +
                b"".join(elem_to_bytes(v) for v in self.output))

    @classmethod
    def from_bytes(cls, b: bytes) -> "OutputData":
        h, off = hash_from_bytes(b, 0)
        view, off = parse_proof(b, off)
        count, off = read_usize(b, off)
        if count != 16:
            raise ValueError("expected an array containing f128::BaseElement of length 16")
        out = []
        for _ in range(count):
            if off + 16 > len(b):
                raise ValueError("truncated output")
            out.append(elem_from_bytes(b[off:off + 16]))
            off += 16
        if off != len(b):
            raise ValueError("trailing bytes after OutputData")
        return cls(h, view.raw, out)
