"""A hash of the library's sources (csrc/ and the public header): stamps the committed PMC profiles, so bench.py can
say whether a profile was taken on the tree it runs (the GPU box has no git history)."""
import hashlib
from pathlib import Path

_PKG = Path(__file__).resolve().parent.parent


def source_hash() -> str:
    h = hashlib.sha256()
    files = sorted(p for p in (_PKG / "csrc").iterdir() if p.suffix in (".hip", ".cpp", ".hpp"))
    files.append(_PKG.parent / "include" / "zkvm_gpu.h")
    for p in files:
        h.update(p.name.encode())
        h.update(p.read_bytes())
    return h.hexdigest()[:16]
