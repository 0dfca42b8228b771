#!/usr/bin/env python3
"""Regenerate the skinny-GEMM register-spill table from hipcc's resource-usage remarks.

kSpillCfg (csrc/kernels/gemm_skinny.hip) and SPILL_CFGS (enterprise_inference_amd/ops/gemm.py)
list the (M-tile count, cfg) instantiations whose weight pipeline does not fit the gfx950
register file (scratch spills); the host never selects them.  ``--write`` patches both."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "csrc", "kernels", "gemm_skinny.hip")
PAT = re.compile(r"gemm_skinny_kernelILi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)ELb([01])ELi(\d+)ELb([01])ELb([01])E")


def main() -> int:
    cmd = [os.environ.get("HIPCC", "hipcc"), "--offload-arch=gfx950", "-O3", "-std=c++17",
           "-munsafe-fp-atomics", "-fgpu-flush-denormals-to-zero",
           "-I" + os.path.join(ROOT, "csrc", "include"),
           "-Rpass-analysis=kernel-resource-usage", "-c", SRC, "-o", "/tmp/_spill.o"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        sys.exit(r.stderr[-3000:])
    cur, spill, seen = None, set(), set()
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            f = PAT.search(m.group(1))
            cur = tuple(int(x) for x in f.groups()) if f else None
            if cur:
                seen.add(cur)
            continue
        if cur is None:
            continue
        m = re.search(r"(ScratchSize \[bytes/lane\]|VGPRs Spill|SGPRs Spill): (\d+)", line)
        if m and int(m.group(2)) > 0:
            spill.add(cur)
    masks = [0] * 9
    # packed-weight variants (cfg bit 6) share their base configuration's bit
    for mt, nt, waves, st, grouped, kc, loader, _packed in spill:
        # grouped (MoE) variants are not table-selected; the 7-wave SwiGLU form (cfg bit 8) has
        # its own fixed M bound in check_shape / gemm.valid
        if grouped or waves in (5, 7):
            continue
        cfg = (nt - 1) | ((waves // 2 - 1) << 1) | ((st - 2) << 2) | (16 if kc == 128 else 0) \
            | (32 if loader else 0)
        masks[mt] |= 1 << cfg
    cpp = "constexpr unsigned long long kSpillCfg[9] = {" + ", ".join(
        hex(m) + "ull" for m in masks) + "};"
    py = "SPILL_CFGS = {" + ", ".join(
        f"{mt}: {tuple(c for c in range(64) if masks[mt] >> c & 1)}" for mt in range(1, 9)) + "}"
    print(f"{len(seen)} instantiations, {len(spill)} spill")
    print(cpp)
    print(py)
    if "--write" in sys.argv:
        s = open(SRC).read()
        s = re.sub(r"constexpr unsigned (long long )?kSpillCfg\[9\] = \{[^}]*\};", cpp, s)
        open(SRC, "w").write(s)
        p = os.path.join(ROOT, "enterprise_inference_amd", "ops", "gemm.py")
        s = open(p).read()
        s = re.sub(r"SPILL_CFGS = \{.*\}\n", py + "\n", s)
        open(p, "w").write(s)
    return 0


if __name__ == "__main__":
    sys.exit(main())
