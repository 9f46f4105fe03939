"""Test-only CPU rehearsal of exchange.OneShotAllGather: the SAME buffer layout and protocols
as comm.hip -- a 256-B head of flags, regions [parity][rank] of 8-byte {word, epoch} granules
(2 x slot_bytes each; k_allgather_granules: workgroup b pushes its share of the words to every
rank and pulls rank b's granules once tagged) for payloads up to 2 KiB, plain slots
[parity][rank] + epoch flags (k_allgather_flags) above, epoch parity -- run by each gloo rank over
shared-memory files standing in for the IPC-mapped device buffers.  Used by
tests/test_exchange.py to check shard placement, ordering and the parity double buffer on
CPU; the device protocol itself runs in tests/test_gpu_xgmi_exchange.py."""
from __future__ import annotations

import os
import time

import numpy as np
import torch
import torch.distributed as dist

HEAD_BYTES = 256   # comm.hip kAgHeadBytes (flags [2][32] u32 of the flag protocol)
GRANULE_MAX = 2048  # comm.hip QZ_AG_GRANULE_MAX_BYTES


class ShmAllGather:
    def __init__(self, group=None, slot_bytes: int = 1 << 12, tag: str = "t"):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.slot_bytes = slot_bytes
        self.nbytes = HEAD_BYTES + 2 * self.world * 2 * slot_bytes + 2 * self.world * slot_bytes  # qz_exchange_bytes
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

    def _region(self, buf, par, q):
        """granules (u64) of rank q's region, parity par, in buf"""
        off = HEAD_BYTES + (par * self.world + q) * 2 * self.slot_bytes
        return buf.numpy()[off:off + 2 * self.slot_bytes].view(np.uint64)

    def accepts(self, inp: torch.Tensor) -> bool:
        n = inp.numel() * inp.element_size()
        return (not inp.is_cuda) and inp.is_contiguous() and n % 16 == 0 and n <= self.slot_bytes

    def _slot(self, buf, par, q):
        """the flag protocol's plain slot of rank q, parity par, in buf"""
        off = HEAD_BYTES + 4 * self.world * self.slot_bytes + (par * self.world + q) * self.slot_bytes
        return buf[off:off + self.slot_bytes]

    def _flags(self, call_epoch, inp, out):
        n = inp.numel() * inp.element_size()
        par = call_epoch & 1
        src = inp.contiguous().reshape(-1).view(torch.uint8)
        for r in range(self.world):                       # push into slot [par][rank] of every rank
            self._slot(self.peers[r], par, self.rank)[:n] = src
        for r in range(self.world):                       # signal
            self.peers[r][:HEAD_BYTES].view(torch.int32)[par * 32 + self.rank] = call_epoch
        flags = self.own[:HEAD_BYTES].view(torch.int32)   # wait (bounded)
        t0 = time.time()
        while any(int(flags[par * 32 + p]) != call_epoch for p in range(self.world)):
            if time.time() - t0 > 60:
                raise TimeoutError("peer flag never arrived")
            time.sleep(1e-4)
        dst = out.reshape(-1).view(torch.uint8)           # unpack, rank-major
        for p in range(self.world):
            dst[p * n:(p + 1) * n] = self._slot(self.own, par, p)[:n]

    def __call__(self, out: torch.Tensor, inp: torch.Tensor) -> None:
        n = inp.numel() * inp.element_size()
        if n > GRANULE_MAX:
            self._flags(self.epoch + 1, inp, out)
            self.epoch += 1
            self.calls += 1
            return
        nw = n // 4
        epoch = self.epoch + 1
        par = epoch & 1
        tag = np.uint64(epoch) << np.uint64(32)
        words = inp.contiguous().reshape(-1).view(torch.int32).numpy().view(np.uint32).astype(np.uint64)
        for b in range(self.world):                    # 1. push: "workgroup" b's share of the words
            w0, w1 = nw * b // self.world, nw * (b + 1) // self.world
            for r in range(self.world):
                self._region(self.peers[r], par, self.rank)[w0:w1] = words[w0:w1] | tag
        dst = out.reshape(-1).view(torch.int32).numpy().view(np.uint32)
        t0 = time.time()
        for b in range(self.world):                    # 2. pull rank b's granules once tagged
            g = self._region(self.own, par, b)[:nw]
            while not np.all((g >> np.uint64(32)) == np.uint64(epoch)):
                if time.time() - t0 > 60:
                    raise TimeoutError("peer granules never arrived")
                time.sleep(1e-4)
                g = self._region(self.own, par, b)[:nw]
            dst[b * nw:(b + 1) * nw] = (g & np.uint64(0xFFFFFFFF)).astype(np.uint32)
        self.epoch = epoch
        self.calls += 1

    def close(self):
        try:
            os.unlink(self.path)
        except OSError:
            pass
