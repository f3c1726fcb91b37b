"""Guards for k_schur's generated MFMA chain (schur_chain.h).

k_schur jumps into the middle of an inline-asm block: s_getpc_b64 returns the address after itself, the chain's
entry is 12 + 8 (n - ns) bytes past it (s_add_u32, s_addc_u32, s_setpc_b64 of 4 bytes each, then n MFMAs of 8
bytes each).  These CPU tests check that (1) the committed header is exactly what tools/gen_schur_chain.py
generates, and (2) in the gfx950 code object hipcc builds from ba_schur.hip, every chain site has that layout, so
every clamped entry ns = 0 .. n lands on an MFMA boundary (ns = 0: the first instruction after the block).
"""
import os
import re
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "slam-robot_amd", "csrc")
LLVM = "/opt/rocm/lib/llvm/bin"
HIPCC = "/opt/rocm/bin/hipcc"


def test_header_matches_generator(tmp_path):
    out = tmp_path / "schur_chain.h"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_schur_chain.py"), "10", "4", str(out)],
                   check=True, capture_output=True)
    committed = open(os.path.join(CSRC, "schur_chain.h")).read()
    assert out.read_text() == committed, "schur_chain.h differs from tools/gen_schur_chain.py's output"


def _disassemble(tmp_path):
    obj, dev = tmp_path / "schur.o", tmp_path / "schur_dev.o"
    subprocess.run([HIPCC, "-O3", "-std=c++17", "-I" + os.path.join(ROOT, "include"), "-I" + CSRC,
                    "--offload-arch=gfx950", "-munsafe-fp-atomics", "--cuda-device-only", "-c",
                    os.path.join(CSRC, "ba_schur.hip"), "-o", str(obj)], check=True, capture_output=True)
    subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", "--input=" + str(obj),
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + str(dev)], check=True,
                   capture_output=True)
    dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", str(dev)], check=True,
                         capture_output=True, text=True).stdout
    ins = []
    for line in dis.splitlines():
        m = re.match(r"\s+(\S.*?)\s*//\s*([0-9A-Fa-f]{12,16}):", line)
        if m:
            ins.append((int(m.group(2), 16), m.group(1)))
    return ins


@pytest.mark.skipif(not (os.path.exists(HIPCC) and shutil.which(os.path.join(LLVM, "llvm-objdump"))),
                    reason="needs the ROCm toolchain (hipcc, llvm-objdump)")
def test_chain_entry_offsets_land_on_mfma_boundaries(tmp_path):
    ins = _disassemble(tmp_path)
    sites = [i for i, (_, t) in enumerate(ins) if t.startswith("s_getpc_b64 s[94:95]")]
    # one site per MFMA wave's chain (four waves), possibly instantiated more than once
    assert len(sites) >= 4, "no asm chain sites found in k_schur"
    seen_n = set()
    for i in sites:
        a_pc, _ = ins[i]
        ret = a_pc + 4   # s_getpc_b64 returns the address of the next instruction
        m = re.match(r"s_min_i32 s93, s93, (\d+)", ins[i - 4][1])
        assert m and ins[i - 5][1].startswith("s_max_i32 s93,") and ins[i - 1][1] == "s_add_u32 s93, s93, 12", \
            "chain site at %#x: clamp sequence not found" % a_pc
        n = int(m.group(1))
        seen_n.add(n)
        assert ins[i + 1] == (ret, "s_add_u32 s94, s94, s93")
        assert ins[i + 2] == (ret + 4, "s_addc_u32 s95, s95, 0")
        assert ins[i + 3] == (ret + 8, "s_setpc_b64 s[94:95]")
        for k in range(n):   # entry for ns = n - k lands on this MFMA
            addr, text = ins[i + 4 + k]
            assert addr == ret + 12 + 8 * k, "MFMA %d of the chain at %#x is not 8-byte spaced" % (k, a_pc)
            assert text.startswith("v_mfma_f64_16x16x4_f64") or text.startswith("v_mfma_f64_4x4x4_4b_f64"), text
        addr, text = ins[i + 4 + n]   # ns = 0: just past the block
        assert addr == ret + 12 + 8 * n and not text.startswith("v_mfma"), text
    assert seen_n == {17, 16}, seen_n   # kSlots of the four waves (TW = 10, CW = 4: 17, 16, 16, 16)
