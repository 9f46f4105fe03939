"""One-shot all-gather of row-split decode outputs over xGMI (the RCCL
replacement the round-2 review asked for).

``OneShotAllGather`` owns this rank's exchange buffer (uncached device memory), maps every
peer's buffer through hipIpc handles (exchanged once over the process group) and runs one
``qz_allgather_oneshot`` launch per all-gather (comm.hip): each rank stores its shard straight
into every peer's buffer as 8-byte {word, epoch} granules, and each rank reads the granules
arriving in its own buffer once their tags carry the call's epoch -- no collective library, no
flag round trip, no host involvement, HIP-graph capturable.

It is selected per model by ``parallel.shard_model_linear4bit(..., gatherer=...)``; anything
it does not take (payloads above its slot, not 16-B multiples, CPU tensors) goes to
``dist.all_gather_into_tensor`` as before.  ``verify`` compares it with RCCL on live data
once at setup (bench.py does, and falls back to RCCL on any mismatch).
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch
import torch.distributed as dist

from . import _lib
from ._lib import check, lib


def _vote(value: int, op, group, device) -> int:
    """MIN/MAX of an int over the group (the tensor on the CPU for gloo, on the GPU for RCCL)."""
    dev = torch.device("cpu") if dist.get_backend(group) == "gloo" else device
    t = torch.tensor([int(value)], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=op, group=group)
    return int(t.item())


class OneShotAllGather:
    """All-gather of up to `slot_bytes` per rank, rank-major output (the order of
    ``dist.all_gather_into_tensor``), through IPC-mapped peer buffers."""

    def __init__(self, group=None, slot_bytes: int = 1 << 16, device: Optional[torch.device] = None):
        if slot_bytes % 16 != 0 or slot_bytes <= 0:
            raise ValueError("slot_bytes must be a positive multiple of 16")
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if self.world > 8:
            raise ValueError("OneShotAllGather supports up to 8 ranks (one MI355X node)")
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.slot_bytes = int(slot_bytes)
        self._own = None
        self._opened = []
        # Every rank reaches the same collectives in the same order whatever fails locally: a
        # local error is carried into the exchange of handles and the MIN vote below, and then
        # raised on EVERY rank (never on one rank while the others wait in a collective).
        err = None
        mine = None
        try:
            nbytes = int(lib.qz_exchange_bytes(self.world, self.slot_bytes))
            own = ctypes.c_void_p()
            check(lib.qz_exchange_alloc(nbytes, ctypes.byref(own)), "qz_exchange_alloc")
            self._own = own
            hsz = int(lib.qz_ipc_handle_size())
            handle = (ctypes.c_char * hsz)()
            check(lib.qz_ipc_get_handle(own, handle), "qz_ipc_get_handle")
            mine = (bytes(handle), self.device.index)
        except Exception as e:  # noqa: BLE001 -- re-raised after the vote
            err = e
        allh = [None] * self.world
        dist.all_gather_object(allh, mine, group=group)
        peers = (ctypes.c_void_p * self.world)()
        if err is None:
            try:
                if any(h is None for h in allh):
                    raise RuntimeError("a peer could not create its exchange buffer")
                for r, (h, dev) in enumerate(allh):
                    if r == self.rank:
                        peers[r] = self._own.value
                        continue
                    check(lib.qz_enable_peer_access(int(dev)), f"qz_enable_peer_access({dev})")
                    p = ctypes.c_void_p()
                    check(lib.qz_ipc_open_handle(ctypes.create_string_buffer(h, hsz), ctypes.byref(p)),
                          f"qz_ipc_open_handle(rank {r})")
                    self._opened.append(p)
                    peers[r] = p.value
            except Exception as e:  # noqa: BLE001 -- re-raised after the vote
                err = e
        self._peers = peers
        self.epoch = torch.zeros(2, dtype=torch.int32, device=self.device)   # epoch, last-finisher ticket
        self.status = torch.zeros(1, dtype=torch.int32, device=self.device)
        if not _vote(err is None, dist.ReduceOp.MIN, group, self.device):
            self.close()
            raise RuntimeError(f"one-shot all-gather setup failed on some rank (here: {err!r})")
        dist.barrier(group=group)   # every rank has mapped every buffer before the first launch

    def accepts(self, inp: torch.Tensor) -> bool:
        n = inp.numel() * inp.element_size()
        return (inp.is_cuda and inp.is_contiguous() and n % 16 == 0 and n <= self.slot_bytes
                and inp.data_ptr() % 16 == 0)

    def __call__(self, out: torch.Tensor, inp: torch.Tensor, mode: int = 0) -> None:
        """out[world * n] <- every rank's inp[n], rank-major (all_gather_into_tensor(out, inp)).
        mode: 0 = by payload size (qz_allgather_oneshot), 1 = flag protocol, 2 = tagged granules."""
        n = inp.numel() * inp.element_size()
        if out.numel() * out.element_size() != self.world * n or not out.is_contiguous():
            raise ValueError("out must be a contiguous tensor of world x inp's bytes")
        args = (inp.data_ptr(), n, out.data_ptr(), self.rank, self.world, self._peers, self._own, self.slot_bytes,
                self.epoch.data_ptr(), self.status.data_ptr())
        if mode:
            check(lib.qz_allgather_oneshot_mode(*args, mode, _lib.stream_of(inp)), "qz_allgather_oneshot_mode")
        else:
            check(lib.qz_allgather_oneshot(*args, _lib.stream_of(inp)), "qz_allgather_oneshot")

    def failed(self) -> bool:
        """True if any launch so far timed out waiting for a peer (synchronises)."""
        return bool(self.status.item())

    def failed_anywhere(self) -> bool:
        """failed() on ANY rank of the group (a collective: every rank must call it)."""
        return bool(_vote(self.failed(), dist.ReduceOp.MAX, self.group, self.device))

    def verify(self, sizes=(256, 2048, 14336), dtype=torch.float16) -> bool:
        """Compare with dist.all_gather_into_tensor on this group for a few payload sizes
        (elements), twice each (both slot parities).  True if every result is identical."""
        ok = True
        g = torch.Generator(device=self.device).manual_seed(1234 + self.rank)
        for n in sizes:
            for _ in range(2):
                x = torch.randn(n, device=self.device, generator=g).to(dtype)
                if not self.accepts(x):
                    continue
                b = torch.empty(self.world * n, device=self.device, dtype=dtype)
                dist.all_gather_into_tensor(b, x, group=self.group)
                for mode in (0, 1, 2):
                    try:   # a local failure must not skip this rank's later collectives
                        a = torch.empty_like(b)
                        self(a, x, mode)
                        ok = ok and bool(torch.equal(a, b))
                    except Exception:  # noqa: BLE001 -- reported by the vote below
                        ok = False
        return bool(_vote(ok and not self.failed(), dist.ReduceOp.MIN, self.group, self.device))

    def warm_graph(self, replays: int = 3) -> bool:
        """Capture and replay a throwaway HIP graph of one call per protocol (collective: every
        rank calls it).  Measured with two processes on one MI355X: the FIRST graph a process
        captures runs its exchanges at ~28 us per call for every replay, whatever the protocol
        or payload, and every later graph at 3.5-4 us; a throwaway graph first removes it
        (`profiles/r4_exchange_first_graph.txt`).  Run before the decode graph is captured.
        Returns the MIN vote of every rank's success (a local failure is voted on, never raised
        on one rank while the others go on): False means no rank may use this gatherer."""
        ok = True
        try:
            n = 256
            x = torch.zeros(n, device=self.device, dtype=torch.float16)
            out = torch.empty(self.world * n, device=self.device, dtype=torch.float16)
            s = torch.cuda.Stream(device=self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(s):
                self(out, x, 1)
                self(out, x, 2)
            torch.cuda.current_stream(self.device).wait_stream(s)
            torch.cuda.synchronize(self.device)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self(out, x, 1)
                self(out, x, 2)
            for _ in range(replays):
                g.replay()
            torch.cuda.synchronize(self.device)
            del g
        except Exception:  # noqa: BLE001 -- reported by the vote below
            ok = False
        try:
            ok = ok and not self.failed()
        except Exception:  # noqa: BLE001
            ok = False
        return bool(_vote(ok, dist.ReduceOp.MIN, self.group, self.device))

    def close(self) -> None:
        for p in self._opened:
            lib.qz_ipc_close_handle(p)
        self._opened = []
        if self._own is not None:
            lib.qz_exchange_free(self._own)
            self._own = None


def all_gather_into(out: torch.Tensor, inp: torch.Tensor, group=None, gatherer=None) -> None:
    """dist.all_gather_into_tensor(out, inp), through `gatherer` when it takes the payload."""
    if gatherer is not None and gatherer.accepts(inp):
        gatherer(out, inp)
    else:
        dist.all_gather_into_tensor(out, inp, group=group)
