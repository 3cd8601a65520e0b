"""Host-side process group of the channel-sharded beamformer: one process per GPU, no torch.

The ranks of a multi-GPU run (launched by `torch.distributed.run`, which only sets RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT) need three host-side services, none on the beamforming data path:
  * the timing bracket: a barrier and a max over ranks (bench.py);
  * the hand-out of the RCCL unique id from rank 0 (bf_comm_create, include/bf.h);
  * a host-memory channel scatter / gather for rehearsals with several ranks on one GPU (RCCL refuses two ranks on
    one device) and for verification.
`HostGroup` provides them over plain TCP: rank 0 listens on MASTER_ADDR:port, every other rank connects once, and
each collective is a star exchange through rank 0 (length-prefixed messages, in call order).  Keeping torch out of
the ranks keeps one HIP runtime (the ROCm release libbf.so is built against) in every process.

The reference has no multi-GPU code; its X-engine index is the only parallel axis (coeff_generator.py:49-53).
"""
import json
import os
import socket
import struct
import time

_HDR = struct.Struct("!Q")


def _send(sock, payload: bytes):
    sock.sendall(_HDR.pack(len(payload)) + payload)


def _recv_exact(sock, n):
    buf = bytearray(n)
    view = memoryview(buf)
    got = 0
    while got < n:
        k = sock.recv_into(view[got:], min(n - got, 1 << 24))
        if k == 0:
            raise ConnectionError("rendezvous peer closed the connection")
        got += k
    return bytes(buf)


def _recv(sock):
    (n,) = _HDR.unpack(_recv_exact(sock, _HDR.size))
    return _recv_exact(sock, n)


def default_port():
    """MASTER_PORT + 1 (torch.distributed.run's own store holds MASTER_PORT), or BF_RDZV_PORT."""
    if os.environ.get("BF_RDZV_PORT"):
        return int(os.environ["BF_RDZV_PORT"])
    return int(os.environ.get("MASTER_PORT", "29531")) + 1


class HostGroup:
    """A star-shaped TCP process group.  All ranks must call the same collectives in the same order."""

    def __init__(self, rank, world, addr=None, port=None, timeout=120.0, op_timeout=900.0):
        self.rank, self.world = int(rank), int(world)
        addr = addr or os.environ.get("MASTER_ADDR", "127.0.0.1")
        port = port if port is not None else default_port()
        self.peers = {}
        self.rejected = []  # rank ids of connections rank 0 dropped (out of range or already registered)
        self.sock = None
        if self.world == 1:
            return
        if self.rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind((addr, port))
            srv.listen(self.world)
            srv.settimeout(timeout)
            try:
                while len(self.peers) < self.world - 1:
                    conn, _ = srv.accept()
                    conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                    conn.settimeout(op_timeout)  # a rank that never joins a collective fails it, not hangs
                    try:
                        (r,) = struct.unpack("!I", _recv_exact(conn, 4))
                    except (OSError, ConnectionError, struct.error):
                        conn.close()
                        continue
                    if not 1 <= r < self.world or r in self.peers:
                        # a stray connection or a repeated rank id: drop it and keep waiting for the real ranks
                        self.rejected.append(r)
                        conn.close()
                        continue
                    self.peers[r] = conn
            finally:
                srv.close()
        else:
            deadline = time.monotonic() + timeout
            while True:
                try:
                    self.sock = socket.create_connection((addr, port), timeout=5.0)
                    break
                except OSError:
                    if time.monotonic() > deadline:
                        raise
                    time.sleep(0.05)
            self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            self.sock.settimeout(op_timeout)
            self.sock.sendall(struct.pack("!I", self.rank))

    # ---- collectives -------------------------------------------------------------------------------------------
    def _gather(self, payload):
        """Rank 0 gets [payload of rank 0, 1, ...]; others None."""
        if self.world == 1:
            return [payload]
        if self.rank == 0:
            return [payload] + [_recv(self.peers[r]) for r in range(1, self.world)]
        _send(self.sock, payload)
        return None

    def _scatter(self, payloads):
        """Rank 0 passes one payload per rank; every rank returns its own."""
        if self.world == 1:
            return payloads[0]
        if self.rank == 0:
            for r in range(1, self.world):
                _send(self.peers[r], payloads[r])
            return payloads[0]
        return _recv(self.sock)

    def barrier(self):
        self._gather(b"")
        self._scatter([b""] * self.world if self.rank == 0 else None)

    def broadcast_bytes(self, data=None):
        """Rank 0's bytes on every rank."""
        return self._scatter([data] * self.world if self.rank == 0 else None)

    def allreduce_max(self, value):
        got = self._gather(struct.pack("!d", float(value)))
        out = None
        if self.rank == 0:
            m = max(struct.unpack("!d", g)[0] for g in got)
            out = [struct.pack("!d", m)] * self.world
        return struct.unpack("!d", self._scatter(out))[0]

    def allreduce_any(self, flag):
        return self.allreduce_max(1.0 if flag else 0.0) > 0

    def scatter_bytes(self, parts=None):
        """Rank 0 passes one bytes-like part per rank; every rank returns its own part."""
        return self._scatter([bytes(p) for p in parts] if self.rank == 0 else None)

    def gather_bytes(self, data):
        """Rank 0 returns every rank's bytes in rank order; others None."""
        return self._gather(bytes(data))

    def gather_json(self, obj):
        """Rank 0 returns every rank's JSON-serialisable object in rank order; others None."""
        got = self._gather(json.dumps(obj).encode())
        return [json.loads(g) for g in got] if got is not None else None

    def close(self):
        for s in list(self.peers.values()) + ([self.sock] if self.sock else []):
            try:
                s.close()
            except OSError:
                pass
        self.peers, self.sock = {}, None
