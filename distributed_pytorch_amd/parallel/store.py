"""Native rendezvous store (csrc/runtime/tcp_store.cpp) with the subset of the torch Store API the
framework uses — ``set`` / ``get`` / ``wait`` / ``add`` — plus a counter barrier.

It lets a job bootstrap RCCL without a torch.distributed process group (``DPA_RENDEZVOUS=native``):
rank 0 serves the store on ``MASTER_ADDR:DPA_STORE_PORT`` (default MASTER_PORT + 1, since torchrun's
agent already owns MASTER_PORT) and every rank connects as a client.  The reference rendezvous at
``tcp://IP:6585`` (main_gather.py:107) maps onto the same store for the CLI launchers.
"""
from __future__ import annotations

import datetime
import struct
from typing import List, Optional

from .. import _ext


class NativeStore:
    def __init__(self, host: str, port: int, rank: int, world: int, timeout_s: float = 600.0):
        C = _ext.require()
        self.rank, self.world = rank, world
        self._server = C.TcpStoreServer("0.0.0.0", port) if rank == 0 else None
        self.port = self._server.port if self._server is not None else port
        self._c = C.TcpStoreClient(host, self.port, float(timeout_s))

    def set(self, key: str, value) -> None:
        self._c.set(key, value if isinstance(value, bytes) else str(value).encode())

    def get(self, key: str) -> bytes:
        return self._c.get(key)

    def wait(self, keys: List[str], timeout: Optional[datetime.timedelta] = None) -> None:
        """Block until every key exists; ``timeout`` bounds the whole wait (default: the store's)."""
        self._c.wait(list(keys), timeout.total_seconds() if timeout is not None else -1.0)

    def delete_key(self, key: str) -> bool:
        return bool(self._c.delete(key))

    def num_keys(self) -> int:
        return int(self._c.num_keys())

    def add(self, key: str, delta: int) -> int:
        return self._c.add(key, int(delta))

    def barrier(self, tag: str) -> None:
        self._c.barrier(tag, self.world)

    def close(self) -> None:
        """Orderly teardown: clients check out, and rank 0 keeps serving until every client has
        (so no client loses the server in the middle of a reply)."""
        if self._c is None:
            return
        if self.world > 1:
            if self.rank != 0:
                if self.add("__closed", 1) == self.world - 1:
                    self.set("__all_closed", b"1")
            else:
                self.get("__all_closed")
        self._c = None
        self._server = None

    def all_max(self, tag: str, value: float) -> float:
        """Max of one float over all ranks (every rank gets it).  The last rank to finish reading
        deletes the tag's keys, so repeated calls leave nothing behind in the store."""
        self.set(f"{tag}/{self.rank}", struct.pack("<d", float(value)))
        m = max(struct.unpack("<d", self.get(f"{tag}/{r}"))[0] for r in range(self.world))
        if self.add(f"{tag}/out", 1) == self.world:
            for r in range(self.world):
                self._c.delete(f"{tag}/{r}")
            self._c.delete(f"{tag}/out")
        return m
