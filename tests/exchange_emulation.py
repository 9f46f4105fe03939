"""Test-only CPU rehearsal of exchange.OneShotAllGather: the SAME buffer layout and protocol
as comm.hip's k_allgather_oneshot (flags [2][32] u32 at the head, slots [parity][rank] of
slot_bytes, epoch parity, push -> signal -> wait -> unpack), run by each gloo rank over
shared-memory files standing in for the IPC-mapped device buffers.  Used by
tests/test_exchange.py to check shard placement, ordering and the parity double buffer on
CPU; the device protocol itself runs in tests/test_gpu_exchange.py."""
from __future__ import annotations

import os
import time

import torch
import torch.distributed as dist

FLAG_BYTES = 256   # comm.hip kAgFlagBytes


class ShmAllGather:
    def __init__(self, group=None, slot_bytes: int = 1 << 12, tag: str = "t"):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.slot_bytes = slot_bytes
        self.nbytes = FLAG_BYTES + 2 * self.world * slot_bytes   # qz_exchange_bytes
        self.path = f"/dev/shm/qz_xchg_{tag}_{os.getpid()}_{self.rank}"
        self.own = torch.from_file(self.path, shared=True, size=self.nbytes, dtype=torch.uint8)
        self.own.zero_()
        paths = [None] * self.world
        dist.all_gather_object(paths, self.path, group=group)
        self.peers = [self.own if r == self.rank else
                      torch.from_file(p, shared=True, size=self.nbytes, dtype=torch.uint8)
                      for r, p in enumerate(paths)]
        self.epoch = 0
        self.calls = 0
        dist.barrier(group=group)

    def accepts(self, inp: torch.Tensor) -> bool:
        n = inp.numel() * inp.element_size()
        return (not inp.is_cuda) and inp.is_contiguous() and n % 16 == 0 and n <= self.slot_bytes

    def __call__(self, out: torch.Tensor, inp: torch.Tensor) -> None:
        n = inp.numel() * inp.element_size()
        epoch = self.epoch + 1
        par = epoch & 1
        slot0 = FLAG_BYTES + par * self.world * self.slot_bytes
        src = inp.contiguous().view(torch.uint8).reshape(-1)
        for r in range(self.world):                       # 1. push into slot [par][rank] of every rank
            off = slot0 + self.rank * self.slot_bytes
            self.peers[r][off:off + n] = src
        for r in range(self.world):                       # 2. signal
            self.peers[r][:FLAG_BYTES].view(torch.int32)[par * 32 + self.rank] = epoch
        flags = self.own[:FLAG_BYTES].view(torch.int32)   # 3. wait (bounded)
        t0 = time.time()
        while any(int(flags[par * 32 + p]) != epoch for p in range(self.world)):
            if time.time() - t0 > 60:
                raise TimeoutError("peer flag never arrived")
            time.sleep(1e-4)
        dst = out.view(torch.uint8).reshape(-1)           # 4. unpack, rank-major
        for p in range(self.world):
            off = slot0 + p * self.slot_bytes
            dst[p * n:(p + 1) * n] = self.own[off:off + n]
        self.epoch = epoch
        self.calls += 1

    def close(self):
        try:
            os.unlink(self.path)
        except OSError:
            pass
