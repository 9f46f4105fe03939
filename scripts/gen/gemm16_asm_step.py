"""Generates quantizations_amd/csrc/gemm16_asm_step.h: ONE 64-deep K-step of k_gemm16_4d's 4-wave
256 x 256 tile (each wave a 128 x 128 quadrant, 128 v_mfma_f32_16x16x32) as a single inline-asm
instruction stream -- every read, DMA, wait and barrier at a fixed MFMA position, and NOTHING the
compiler adds (hipcc's waitcnt pass inserted conservative lgkmcnt waits at the loop header and around
the pinned regions of the HIP form).  Schedules:
  SPLIT  kGemm4Split (gemm.hip): the buffer just read released per operand, waits + barriers after
         MFMAs 21, 51 (lgkmcnt(0)) and 92 (vmcnt(13)), the next step's reads spread over the rest;
  L0/L1  the same release structure with each barrier one MFMA after its wait, and the two event
         orders the library's MT256x256x64 kernel alternates between waves on even and odd SIMDs.
W fragment offsets: NAT (fragment j = rows 16 j .. 16 j + 15 of the wave's 128) or PERM (rows
32 (j / 2) + 8 (fr / 4) + 4 (j % 2) + fr % 4: a lane's accumulators of fragments 2J, 2J + 1 hold 8
consecutive output rows -- k_gemm16_4d's S & 2 register epilogue).

Operands (GCC numbering): %0..%63 the accumulators acc[j][i] (j = n / 8, i = n % 8; AGPR quads),
%64..%71 X fragments of k-half 0 (xa[i]), %72..%79 W k-half 0 (wa[j]), %80..%87 X k-half 1 (xb[i]),
%88..%95 W k-half 1 (wb[j]) -- all read-write; inputs %96 / %97 the LDS bases of this step's X / W
k-half-1 fragments, %98 / %99 of step s + 1's X / W k-half-0 fragments, %100..%107 the X DMA offsets,
%108..%115 the W DMA offsets, %116 / %117 the X / W buffer descriptors, %118 the step's byte offset
along K, %119 the LDS destination of this wave's first X piece in the buffer being refilled; DUAL
(L0 and L1 in ONE statement, so both orders share one register assignment) takes %120, the low bit
of the wave's SIMD, and branches on it.  *_FIRST (the persistent k_gemm16_4q's first step of a
tile): the k-half 0 MFMAs take 0 as the accumulator input (the previous tile's sums are stored).
   python scripts/gen/gemm16_asm_step.py > quantizations_amd/csrc/gemm16_asm_step.h"""


def table(rx1, rw1, dx, dw, rx0, rw0, waits):
    ev = {}
    for i in range(8):
        for kind, pos in (("rx1", rx1), ("rw1", rw1), ("dx", dx), ("dw", dw), ("rx0", rx0), ("rw0", rw0)):
            ev.setdefault(pos[i], []).append((kind, i))
    for c, kind in waits:
        ev.setdefault(c, []).append((kind, 0))
    return ev


SCHEDS = {
    "SPLIT": table([1, 3, 5, 7, 9, 11, 13, 15], [25, 28, 31, 34, 37, 39, 41, 43], [23, 26, 29, 32, 35, 53, 56, 59],
                   [62, 65, 86, 88, 90, 97, 101, 125], [94, 95, 96, 98, 99, 103, 104, 105],
                   [106, 107, 110, 113, 115, 118, 121, 124],
                   [(21, "lgkm"), (21, "bar"), (51, "lgkm"), (51, "bar"), (92, "vm13"), (92, "bar"), (127, "lgkm")]),
    "L0": table([1, 3, 5, 7, 9, 11, 13, 15], [25, 28, 31, 34, 37, 39, 41, 43], [23, 26, 29, 32, 35, 53, 56, 59],
                [62, 65, 86, 88, 90, 97, 101, 125], [94, 95, 96, 98, 99, 103, 104, 105],
                [106, 107, 110, 113, 115, 118, 121, 124],
                [(21, "lgkm"), (22, "bar"), (51, "lgkm"), (52, "bar"), (92, "vm13"), (93, "bar"), (127, "lgkm")]),
    "L1": table([1, 3, 5, 7, 9, 11, 13, 15], [23, 26, 29, 32, 35, 39, 41, 43], [24, 27, 30, 33, 36, 54, 57, 60],
                [63, 66, 85, 87, 89, 96, 100, 124], [94, 95, 97, 98, 99, 103, 104, 105],
                [106, 107, 110, 113, 115, 118, 121, 123],
                [(21, "lgkm"), (22, "bar"), (51, "lgkm"), (52, "bar"), (92, "vm13"), (93, "bar"), (127, "lgkm")]),
}
DMAS = [("dx", c) for c in range(8)] + [("dw", c) for c in range(8)]   # issue order
DMAS_WF = [("dw", c) for c in range(8)] + [("dx", c) for c in range(8)]


def m0_for(kind, c):
    return 4096 * c + (32768 if kind == "dw" else 0)


def w_off(j, perm):
    return (4096 * (j >> 1) + 512 * (j & 1)) if perm else 2048 * j


def wfirst(ev):
    """The same slots with the operands' k-half 1 reads and refill DMAs swapped: W's fragments read
    first, so the W image is released (and refilled) first, X's after the second wait."""
    sw = {"rx1": "rw1", "rw1": "rx1", "dx": "dw", "dw": "dx"}
    return {c: [(sw.get(k, k), i) for k, i in es] for c, es in ev.items()}


def stream(ev, perm, t, first=False, dmas=None):
    DMAS = dmas or globals()["DMAS"]
    order = sorted((c, e) for c, es in ev.items() for e in es if e[0] in ("dx", "dw"))
    assert [e for _, e in order] == DMAS, order
    dmacount = sum(1 for c, es in ev.items() for e in es if e[0] in ("dx", "dw") and c < 92)
    vmw = [e[0] for es in ev.values() for e in es if e[0] in ("vm13", "vm16")]
    assert dmacount == (16 if vmw == ["vm16"] else 13), (dmacount, vmw)
    out = [f"s_add_u32 m0, %119, {m0_for(*DMAS[0])}"]
    d = 0
    for n in range(128):
        kk, m = n // 64, n % 64
        j, i = m // 8, m % 8
        a = 72 + j if kk == 0 else 88 + j         # W fragment operand
        b = 64 + i if kk == 0 else 80 + i         # X fragment operand
        # first: a tile's step 0 -- the k-half 0 MFMAs start from 0, not from the accumulator
        out.append(f"v_mfma_f32_16x16x32_{t} %{m}, %{a}, %{b}, {0 if first and kk == 0 else '%' + str(m)}")
        for kind, idx in sorted(ev.get(n + 1, []), key=lambda e: ("lgkm", "vm13", "vm16", "bar").index(e[0])
                                if e[0] in ("lgkm", "vm13", "vm16", "bar") else -1):
            if kind == "rx1":
                out.append(f"ds_read_b128 %{80 + idx}, %96 offset:{2048 * idx}")
            elif kind == "rw1":
                out.append(f"ds_read_b128 %{88 + idx}, %97 offset:{w_off(idx, perm)}")
            elif kind == "rx0":
                out.append(f"ds_read_b128 %{64 + idx}, %98 offset:{2048 * idx}")
            elif kind == "rw0":
                out.append(f"ds_read_b128 %{72 + idx}, %99 offset:{w_off(idx, perm)}")
            elif kind in ("dx", "dw"):
                assert DMAS[d] == (kind, idx)
                voff = 100 + idx if kind == "dx" else 108 + idx
                rs = 116 if kind == "dx" else 117
                out.append(f"buffer_load_dwordx4 %{voff}, %{rs}, %118 offen lds")
                d += 1
                if d < 16:   # the next DMA's LDS destination, at least one MFMA ahead of it
                    out.append(f"s_add_u32 m0, %119, {m0_for(*DMAS[d])}")
            elif kind == "lgkm":
                out.append("s_waitcnt lgkmcnt(0)")
            elif kind == "vm13":
                out.append("s_waitcnt vmcnt(13)")
            elif kind == "vm16":
                out.append("s_waitcnt vmcnt(16)")
            elif kind == "bar":
                out.append("s_barrier")
    assert d == 16
    return out


print("// GENERATED by scripts/gen/gemm16_asm_step.py -- do not edit.  One K-step of k_gemm16_4d<..., S & 64>")
print("// as one hand-ordered instruction stream; operands and schedules: see the generator's docstring.")
for sname in SCHEDS:
    for perm in (False, True):
        for t in ("f16", "bf16"):
            print(f"#define QZ_GEMM16_ASM_{sname}_{'PERM' if perm else 'NAT'}_{t.upper()} \\")
            for ln in stream(SCHEDS[sname], perm, t):
                print(f'  "{ln}\\n\\t" \\')
            print('  ""')
for perm in (False, True):
    for t in ("f16", "bf16"):
        for first in ((False, True) if perm else (False,)):
            w = ('PERM' if perm else 'NAT') + ('_FIRST' if first else '')
            print(f"#define QZ_GEMM16_ASM_DUAL_{w}_{t.upper()} \\")
            body = (["s_cmp_lg_u32 %120, 0", "s_cbranch_scc1 .Lqz_g16_l1_%=",]
                    + stream(SCHEDS["L0"], perm, t, first) + ["s_branch .Lqz_g16_end_%=", ".Lqz_g16_l1_%=:"]
                    + stream(SCHEDS["L1"], perm, t, first) + [".Lqz_g16_end_%=:"])
            for ln in body:
                print(f'  "{ln}\\n\\t" \\')
            print('  ""')
for t in ("f16", "bf16"):
    for first in (False, True):
        w = 'PERM' + ('_FIRST' if first else '')
        print(f"#define QZ_GEMM16_ASM_DUALW_{w}_{t.upper()} \\")
        body = (["s_cmp_lg_u32 %120, 0", "s_cbranch_scc1 .Lqz_g16_l1_%=",]
                + stream(wfirst(SCHEDS["L0"]), True, t, first, DMAS_WF)
                + ["s_branch .Lqz_g16_end_%=", ".Lqz_g16_l1_%=:"]
                + stream(wfirst(SCHEDS["L1"]), True, t, first, DMAS_WF) + [".Lqz_g16_end_%=:"])
        for ln in body:
            print(f'  "{ln}\\n\\t" \\')
        print('  ""')
for t in ("f16", "bf16"):
    print(f"#define QZ_GEMM16_ASM_SPLIT_PERM_FIRST_{t.upper()} \\")
    for ln in stream(SCHEDS["SPLIT"], True, t, True):
        print(f'  "{ln}\\n\\t" \\')
    print('  ""')
