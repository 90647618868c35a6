"""A small torch-free process group over TCP for the host side of a multi-process run.

One process per GPU never needs torch: the library brings its own HIP runtime and RCCL (native.runtime_info()), and
what the host processes still have to agree on goes through this group --

  * the rendezvous (rank 0's listening port; under torchrun published through a file in the temp directory, keyed by
    MASTER_ADDR / MASTER_PORT / TORCHELASTIC_RUN_ID, because torchrun's agent holds MASTER_PORT itself);
  * barriers and the max over ranks of the bench's timed region (bench.py);
  * the 128-byte RCCL unique id, broadcast from rank 0 (zk_comm_unique_id -> zk_comm_create_rccl);
  * the exchange callback of zk_comm_create_host (exchange_fn(): all-to-all and all-gather of host buffers), the
    transport of the one-rank-per-process tests and of the bench's single-GPU rehearsal of the multi-GPU flow.

Every pair of ranks holds its own socket (full mesh).  A collective sends to every peer on one thread and receives
from every peer on another, so no pair of large transfers can wait on each other.  All ranks must call the
collectives in the same order (as with any process group).
"""
from __future__ import annotations

import ctypes as C
import os
import secrets
import socket
import struct
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor

from . import native

_HDR = struct.Struct("<Q")


def _recv_exact(s: socket.socket, n: int) -> bytearray:
    buf = bytearray(n)
    view = memoryview(buf)
    got = 0
    while got < n:
        k = s.recv_into(view[got:], n - got)
        if k == 0:
            raise ConnectionError("host group: peer closed the connection")
        got += k
    return buf


def _send_msg(s: socket.socket, payload) -> None:
    s.sendall(_HDR.pack(len(payload)))
    if len(payload):
        s.sendall(payload)


def _recv_msg(s: socket.socket) -> bytes:
    (n,) = _HDR.unpack(bytes(_recv_exact(s, _HDR.size)))
    return bytes(_recv_exact(s, n)) if n else b""


def _require_local(addr: str) -> None:
    """Every rank runs on the MASTER_ADDR host (the rendezvous file lives in its temp directory and every listener
    binds that address): fail at once, with the reason, instead of retrying to the deadline on another host."""
    try:
        with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as t:
            t.bind((addr, 0))
    except OSError as e:
        raise RuntimeError(f"host group: MASTER_ADDR={addr} is not an address of this host ({e}); the torch-free host "
                           f"group serves single-node runs only (one process per GPU of one node)") from None


def _rdzv_file(addr: str, key: str) -> str:
    safe = "".join(ch if ch.isalnum() else "_" for ch in f"{addr}-{key}")
    return os.path.join(tempfile.gettempdir(), f"zkvm-hostgroup-{safe}")


class HostGroup:
    def __init__(self, rank: int, world: int, addr: str = "127.0.0.1", port: int | None = None,
                 rdzv_key: str | None = None, timeout: float = 300.0):
        """rank 0 listens on `port` (or an ephemeral port published through the rendezvous file named by rdzv_key);
        the other ranks connect to it, then every pair of ranks opens its own connection."""
        if not (0 <= rank < world):
            raise ValueError(f"rank {rank} outside world {world}")
        self.rank, self.world, self.addr = rank, world, addr
        self.peers: dict[int, socket.socket] = {}
        self._pool = ThreadPoolExecutor(max_workers=max(2, 2 * (world - 1))) if world > 1 else None
        if world == 1:
            return
        _require_local(addr)
        deadline = time.monotonic() + timeout
        # every rank's own listener for the mesh connections of the ranks above it, on an ephemeral port -- created
        # only once rank 0's hub is bound (rank 0: after binding it; the others: after reaching it), so that no
        # listener can take an explicitly given hub port first
        if rank == 0:
            hub = self._bind_hub(addr, port, world, deadline)
            hub.settimeout(timeout)
            lst = socket.create_server((addr, 0))
            lst.settimeout(timeout)
            my_port = lst.getsockname()[1]
            nonce = secrets.token_hex(8)
            path = None
            if port is None:
                path = _rdzv_file(addr, rdzv_key or "default")
                tmp = f"{path}.{os.getpid()}"
                with open(tmp, "w") as f:
                    f.write(f"{hub.getsockname()[1]} {nonce}\n")
                os.replace(tmp, path)
            self._rdzv_path = path
            conns, ports = {}, {0: my_port}
            while len(conns) < world - 1:
                c, _ = hub.accept()
                c.settimeout(timeout)
                try:
                    # greet first: a rank that reached a stale port (a rendezvous file of an earlier run) learns at
                    # once that no hub of this run answers there, and re-reads the file
                    _send_msg(c, f"zkhub {nonce}".encode())
                    r, w, p, tok = _recv_msg(c).decode().split()
                except Exception:
                    c.close()
                    continue
                if int(w) != world or (port is None and tok != nonce) or not (0 < int(r) < world) or int(r) in conns:
                    c.close()
                    continue
                conns[int(r)] = c
                ports[int(r)] = int(p)
            table = " ".join(str(ports[r]) for r in range(world)).encode()
            for r, c in conns.items():
                _send_msg(c, table)
            hub.close()
            if path:
                try:
                    os.unlink(path)
                except OSError:
                    pass
            self.peers.update(conns)  # the hub connections are rank 0's mesh links
        else:
            c, table, lst = self._connect_hub(addr, port, rdzv_key, deadline, timeout)
            self.peers[0] = c
            # mesh: rank r connects to every rank s in (0, r) and accepts from every rank above it
            for s in range(1, rank):
                c = socket.create_connection((addr, table[s]), timeout=timeout)
                _send_msg(c, str(rank).encode())
                self.peers[s] = c
            while len(self.peers) < world - 1:
                c, _ = lst.accept()
                c.settimeout(timeout)
                s = int(_recv_msg(c).decode())
                self.peers[s] = c
        lst.close()
        for c in self.peers.values():
            c.settimeout(None)
            c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)

    @staticmethod
    def _bind_hub(addr, port, world, deadline):
        """Rank 0's hub socket on `port` (None: an ephemeral one).  A given port that is briefly taken (another
        process's outgoing connection can hold it as its ephemeral port for a moment) is retried until the deadline."""
        while True:
            try:
                return socket.create_server((addr, port or 0), backlog=world)
            except OSError as e:
                if port is None or e.errno not in (98, 48) or time.monotonic() > deadline:  # EADDRINUSE
                    raise
                time.sleep(0.05)

    def _connect_hub(self, addr, port, rdzv_key, deadline, timeout):
        """Connect to rank 0's hub, create this rank's mesh listener, and wait for the table of every rank's mesh
        port; returns (hub connection, table, listener).  Retried while rank 0 is not listening yet or the rendezvous
        file is a stale one (refused, or closed by a hub with another nonce)."""
        last, lst = None, None
        while time.monotonic() < deadline:
            tok, hub_port = "-", port
            if port is None:
                try:
                    with open(_rdzv_file(addr, rdzv_key or "default")) as f:
                        hub_port, tok = f.read().split()
                    hub_port = int(hub_port)
                except (OSError, ValueError):
                    time.sleep(0.05)
                    continue
            c, greeted = None, False
            try:
                c = socket.create_connection((addr, hub_port), timeout=5.0)
                c.settimeout(5.0)  # the hub greets at once; a silent listener is not this run's hub
                hello = _recv_msg(c).decode().split()
                if len(hello) != 2 or hello[0] != "zkhub" or (port is None and hello[1] != tok):
                    raise ConnectionError("host group: not this run's hub")
                if lst is None:
                    lst = socket.create_server((addr, 0))
                    lst.settimeout(timeout)
                _send_msg(c, f"{self.rank} {self.world} {lst.getsockname()[1]} {tok}".encode())
                greeted = True  # (a timeout from here on is the other ranks', not a stale port)
                c.settimeout(max(1.0, deadline - time.monotonic()))
                table = [int(x) for x in _recv_msg(c).decode().split()]
                if len(table) != self.world:
                    raise ConnectionError(f"host group: a table of {len(table)} ranks")
                return c, table, lst
            except socket.timeout as e:
                if greeted:
                    raise TimeoutError(f"host group: rank {self.rank} waited for the other ranks past the deadline")
                last = e  # no greeting within 5 s: a stale rendezvous file's port; read the file again
                if c is not None:
                    c.close()
                time.sleep(0.05)
            except (OSError, ConnectionError, ValueError) as e:
                last = e
                if c is not None:
                    c.close()
                time.sleep(0.05)
        if lst is not None:
            lst.close()
        raise TimeoutError(f"host group: rank {self.rank} could not reach rank 0 ({last})")

    @classmethod
    def from_env(cls, timeout: float = 300.0) -> "HostGroup":
        """The torchrun environment (RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT, TORCHELASTIC_RUN_ID): rank 0
        listens on an ephemeral port published through the rendezvous file (torchrun's agent holds MASTER_PORT)."""
        rank, world = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))
        addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
        key = f"{os.environ.get('MASTER_PORT', '0')}-{os.environ.get('TORCHELASTIC_RUN_ID', 'none')}"
        return cls(rank, world, addr=addr, rdzv_key=key, timeout=timeout)

    # ---- collectives (every rank, same order)
    def _exchange(self, out: dict) -> dict:
        """Send out[s] to every peer s and receive one message from each; returns {peer: bytes}."""
        peers = sorted(self.peers)
        sends = [self._pool.submit(_send_msg, self.peers[s], out[s]) for s in peers]
        recvs = {s: self._pool.submit(_recv_msg, self.peers[s]) for s in peers}
        got = {s: f.result() for s, f in recvs.items()}
        for f in sends:
            f.result()
        return got

    def all_gather(self, payload: bytes) -> list:
        if self.world == 1:
            return [bytes(payload)]
        got = self._exchange({s: payload for s in self.peers})
        got[self.rank] = bytes(payload)
        return [got[r] for r in range(self.world)]

    def all_to_all(self, chunks: list) -> list:
        """chunks[s] goes to rank s; returns the chunk every rank sent to this one, by source rank."""
        if self.world == 1:
            return [bytes(chunks[0])]
        got = self._exchange({s: chunks[s] for s in self.peers})
        got[self.rank] = bytes(chunks[self.rank])
        return [got[r] for r in range(self.world)]

    def barrier(self) -> None:
        self.all_gather(b"")

    def max(self, value: float) -> float:
        return max(struct.unpack("<d", b)[0] for b in self.all_gather(struct.pack("<d", float(value))))

    def broadcast(self, payload: bytes | None, src: int = 0) -> bytes:
        vals = self.all_gather(payload if self.rank == src else b"")
        return vals[src]

    def exchange_fn(self):
        """A native.EXCHANGE_FN for zk_comm_create_host over this group (keep it alive with the communicator)."""
        world = self.world

        def fn(_ctx, op, send, recv, nbytes):
            try:
                if nbytes:
                    if op == native.XCHG_ALL_TO_ALL:
                        src = C.string_at(send, nbytes * world)
                        parts = self.all_to_all([src[k * nbytes:(k + 1) * nbytes] for k in range(world)])
                    elif op == native.XCHG_ALL_GATHER:
                        parts = self.all_gather(C.string_at(send, nbytes))
                    else:
                        return 2
                    for k, b in enumerate(parts):
                        if len(b) != nbytes:
                            return 3
                        C.memmove(recv + k * nbytes, b, nbytes)
                elif op not in (native.XCHG_ALL_TO_ALL, native.XCHG_ALL_GATHER):
                    return 2
                return 0
            except Exception as e:  # an exception must not unwind through the C frames
                import sys
                print(f"zk exchange callback: {type(e).__name__}: {e}", file=sys.stderr)
                return 1

        return native.EXCHANGE_FN(fn)

    def close(self) -> None:
        for c in self.peers.values():
            try:
                c.close()
            except OSError:
                pass
        self.peers = {}
        if self._pool is not None:
            self._pool.shutdown(wait=False)
            self._pool = None
