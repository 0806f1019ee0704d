"""hostcomm -- rank-to-rank host messages for bench.py and the GPU tests.

One process per GPU (torch.distributed.run sets RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT).  The library's data path uses RCCL itself
(exchange.cpp); what the harness needs on the host is tiny -- a barrier, a
max / min / sum of a few doubles, and rank 0's 128-byte RCCL unique id --
so it goes over plain TCP sockets in a star around rank 0.  No torch is
imported: a torch ROCm wheel carries its own HIP runtime, and a process that
loads it beside libipo_hip.so's (/opt/rocm) holds two runtimes, whose
teardown at exit faulted in round 2 (VERDICT.md "What's weak" 5).

Rank 0 listens on MASTER_PORT + port_offset (the launcher's own store
holds MASTER_PORT); every other rank connects, retrying until `timeout`.
Operations are collective: every rank calls them in the same order.
"""
from __future__ import annotations

import os
import socket
import struct
import time

import numpy as np

OPS = {"sum": np.add, "max": np.maximum, "min": np.minimum}


def _recv(sock: socket.socket, n: int) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("hostcomm: peer closed")
        buf += chunk
    return bytes(buf)


def _send_msg(sock: socket.socket, data: bytes) -> None:
    sock.sendall(struct.pack("<Q", len(data)) + data)


def _recv_msg(sock: socket.socket) -> bytes:
    (n,) = struct.unpack("<Q", _recv(sock, 8))
    return _recv(sock, n)


class HostComm:
    """Star allreduce / broadcast over TCP; a no-op for world == 1."""

    def __init__(self, rank: int | None = None, world: int | None = None, addr: str | None = None,
                 port: int | None = None, port_offset: int = 17, timeout: float = 300.0):
        self.rank = int(os.environ.get("RANK", "0")) if rank is None else rank
        self.world = int(os.environ.get("WORLD_SIZE", "1")) if world is None else world
        self.peers: list[socket.socket] = []
        self.sock: socket.socket | None = None
        if self.world <= 1:
            return
        addr = addr or os.environ.get("MASTER_ADDR", "127.0.0.1")
        port = (port or int(os.environ.get("MASTER_PORT", "29500"))) + port_offset
        if self.rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind((addr, port))
            srv.listen(self.world)
            srv.settimeout(timeout)
            peers = {}
            while len(peers) < self.world - 1:
                c, _ = srv.accept()
                c.settimeout(None)    # the timeout bounds the rendezvous, not later collectives
                c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                (r,) = struct.unpack("<i", _recv(c, 4))
                peers[r] = c
            srv.close()
            self.peers = [peers[r] for r in range(1, self.world)]
        else:
            t0 = time.time()
            while True:
                try:
                    s = socket.create_connection((addr, port), timeout=timeout)
                    break
                except OSError:
                    if time.time() - t0 > timeout:
                        raise
                    time.sleep(0.05)
            # the connect timeout must not stay on the socket: a collective in
            # which rank 0 is busy longer (setup of a large LP, rank-0-only
            # bench legs) would raise socket.timeout here
            s.settimeout(None)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            s.sendall(struct.pack("<i", self.rank))
            self.sock = s

    # ------------------------------------------------------------ collectives
    def allreduce(self, a: np.ndarray, op: str = "sum") -> np.ndarray:
        """In-place reduction of a float64 array over all ranks (rank order)."""
        a = np.asarray(a)
        if self.world <= 1:
            return a
        if self.rank == 0:
            acc = a.astype(np.float64).copy()
            for p in self.peers:
                v = np.frombuffer(_recv_msg(p), np.float64).reshape(acc.shape)
                acc = OPS[op](acc, v)
            data = acc.tobytes()
            for p in self.peers:
                _send_msg(p, data)
        else:
            _send_msg(self.sock, np.ascontiguousarray(a, np.float64).tobytes())
            acc = np.frombuffer(_recv_msg(self.sock), np.float64).reshape(a.shape)
        a[...] = acc
        return a

    def reduce_scalar(self, v: float, op: str) -> float:
        return float(self.allreduce(np.array([float(v)]), op)[0])

    def barrier(self) -> None:
        self.allreduce(np.zeros(1), "sum")

    def bcast_bytes(self, data: bytes | None) -> bytes:
        """Rank 0's bytes on every rank."""
        if self.world <= 1:
            return data
        if self.rank == 0:
            for p in self.peers:
                _send_msg(p, data)
            return data
        return _recv_msg(self.sock)

    def close(self) -> None:
        for s in self.peers + ([self.sock] if self.sock else []):
            try:
                s.close()
            except OSError:
                pass
        self.peers, self.sock = [], None
