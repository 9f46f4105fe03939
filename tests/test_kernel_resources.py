"""CPU: register budgets of the built decode kernels, read from libquantizations.so's gfx950 code
objects (no GPU needed).

Round 4 shipped, for one session, a straight-line GEMV body that hipcc compiled to 260 VGPRs (the
excess spilled into AGPRs): one wave per SIMD, and Llama-3-70B decode fell from 91.9 to 57.9 tok/s
while every parity test stayed green (profiles/r4_bench_70b_two_step_regression.txt).  This test
fails on that class of regression: every decode GEMV instantiation for 16-bit activations with up
to 4 rows per wave must fit the 256 architectural VGPRs with no AGPR spill and no scratch.
"""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "quantizations_amd", "libquantizations.so")
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _tools_ok():
    return (os.path.exists(LIB) and shutil.which("c++filt") is not None
            and all(os.path.exists(os.path.join(LLVM, t)) for t in ("llvm-objcopy", "clang-offload-bundler",
                                                                    "llvm-readelf")))


def kernel_resources(lib=LIB):
    """{demangled kernel name: (vgpr_count, agpr_count, private_segment_fixed_size, sgpr_spill_count,
    vgpr_spill_count)} for every gfx950 kernel in the library's offload bundles."""
    out = {}
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section", f".hip_fatbin={fat}", lib, os.devnull],
                       check=True, capture_output=True)
        blob = open(fat, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), blob)]
        names = []
        for i, st in enumerate(starts):
            en = starts[i + 1] if i + 1 < len(starts) else len(blob)
            b, co = os.path.join(d, f"b{i}.bin"), os.path.join(d, f"co{i}.o")
            with open(b, "wb") as f:
                f.write(blob[st:en])
            r = subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--type=o",
                                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={b}", f"--output={co}",
                                "--unbundle"], capture_output=True)
            if r.returncode != 0 or not os.path.getsize(co):
                continue
            notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], capture_output=True,
                                   text=True, check=True).stdout
            for ent in notes.split("  - .agpr_count:")[1:]:
                agpr = int(ent.split("\n")[0].strip())
                name = re.search(r"\.name:\s+(\S+)", ent).group(1)
                vgpr = int(re.search(r"\.vgpr_count:\s+(\d+)", ent).group(1))
                priv = int(re.search(r"\.private_segment_fixed_size:\s+(\d+)", ent).group(1))
                ssp = re.search(r"\.sgpr_spill_count:\s+(\d+)", ent)
                vsp = re.search(r"\.vgpr_spill_count:\s+(\d+)", ent)
                names.append(name)
                out[name] = (vgpr, agpr, priv, int(ssp.group(1)) if ssp else 0, int(vsp.group(1)) if vsp else 0)
        dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True,
                             check=True).stdout.split("\n")
    return {dm: out[n] for n, dm in zip(names, dem)}


def _targs(demangled):
    m = re.search(r"<(.*)>\(", demangled)
    return [a.strip() for a in m.group(1).split(",")] if m else []


@pytest.mark.skipif(not _tools_ok(), reason="libquantizations.so or the ROCm LLVM tools are missing")
def test_decode_gemv_kernels_fit_without_spills():
    res = kernel_resources()
    checked, bad = 0, []
    for name, (vgpr, agpr, priv, ssp, vsp) in res.items():
        base = name.split("<")[0].replace("void ", "").strip()
        a = _targs(name)
        # every decode kernel's template starts <DQ, DT, R, ...>
        if base not in ("qz::k_gemv_4bit", "qz::k_gemv_4bit_grouped", "qz::k_gemv_4bit_pair") or len(a) < 4:
            continue
        dt, r = int(a[1]), int(a[2])
        if dt not in (0, 1) or r > 4:   # 16-bit activations (F16 = 0, BF16 = 1), up to 4 rows per wave
            continue
        checked += 1
        if agpr > 0 or priv > 0 or vgpr > 256 or vsp or ssp:
            bad.append((vgpr, agpr, priv, ssp, vsp, name))
    assert checked > 50, f"only {checked} decode GEMV kernels found in the code objects"
    assert not bad, "decode GEMV kernels that spill:\n" + "\n".join(map(str, sorted(bad, reverse=True)[:20]))


@pytest.mark.skipif(not _tools_ok(), reason="libquantizations.so or the ROCm LLVM tools are missing")
def test_product_decode_picks_keep_two_waves_per_simd():
    """The instantiations the Llama-3-8B decode launches (rocprofv3 census, profiles/r4_decode_anatomy.txt)
    stay within 256 VGPRs: at least two waves per SIMD."""
    res = kernel_resources()
    picks = [
        "qz::k_gemv_4bit_pair<true, 0, 4, true, true, true, true, true>",          # gate/up + SiLU + norm
        "qz::k_gemv_4bit<true, 0, 2, 1, 8, true, true, true, false, 0>",           # down_proj + residual
        "qz::k_gemv_4bit_grouped<true, 0, 2, 1, true, true, true, true>",          # q/k/v + norm
        "qz::k_gemv_4bit<true, 0, 2, 1, 4, true, true, false, true, 0>",           # o_proj + residual
    ]
    for p in picks:
        hits = [v for k, v in res.items() if p in k]
        assert hits, f"{p} not in the library"
        vgpr, agpr, priv, ssp, vsp = hits[0]
        assert vgpr <= 256 and agpr == 0 and priv == 0 and ssp == 0 and vsp == 0, (p, vgpr, agpr, priv, ssp, vsp)
