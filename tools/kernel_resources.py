"""Register / LDS / scratch report of the hot kernels (gfx950), from the compiler's own
metadata: python tools/kernel_resources.py [source.hip ...]
Compiles each source device-only to assembly (hipcc -S, the library's flags) and prints, per
kernel matching the hot-path names, VGPRs, spilled VGPRs, static LDS and the private
(scratch) segment -- a spill or a scratch segment in a hot kernel is a regression to catch
before a GPU run (scratch can also throttle how many waves a launch gets)."""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CS = os.path.join(ROOT, "fm-returnprediction_amd", "csrc")
HOT = ("select_pair_hk_kernelILi40", "select_pair_kernelILi40", "select_fixup_universe_kernelILi20",
       "select_fixup_kernelILi20", "select_long_hk_kernelILi40", "universe_kernelILi20",
       "gram_kernelILi1ELi15ELi3ELb1", "gram_kernelILi1ELi15ELi3ELb0", "solve16_kernel", "ts_fused_kernel",
       "rolling_std_kernel", "firm_chars_kernel", "split_planes_kernel")


def report(src):
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "k.s")
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
               "-I" + os.path.join(ROOT, "include"), "-I" + CS, "--offload-device-only", "-S", "-o", out, src]
        subprocess.run(cmd, check=True, capture_output=True)
        s = open(out).read()
    rows = []
    for m in re.finditer(r"- \.agpr_count:.*?\.name:\s+(\S+).*?\.vgpr_count:\s+(\d+)\s+\.vgpr_spill_count:\s+(\d+)",
                         s, re.S):
        blk = m.group(0)
        name = m.group(1)
        if not any(h in name for h in HOT):
            continue
        lds = re.search(r"\.group_segment_fixed_size:\s+(\d+)", blk)
        priv = re.search(r"\.private_segment_fixed_size:\s+(\d+)", blk)
        rows.append((name, int(m.group(2)), int(m.group(3)), int(lds.group(1)) if lds else -1,
                     int(priv.group(1)) if priv else -1))
    return rows


def main():
    srcs = sys.argv[1:] or [os.path.join(CS, f) for f in ("fm_select.hip", "fm_gram.hip", "fm_solve.hip",
                                                           "fm_ts.hip", "fm_chars.hip", "fm_elem.hip")]
    bad = 0
    for src in srcs:
        for name, vgpr, spill, lds, priv in report(src):
            flag = "  <-- spills / scratch" if spill or priv > 0 else ""
            bad += bool(flag)
            print(f"{os.path.basename(src):14s} {name[:64]:64s} vgpr {vgpr:3d} spill {spill:3d} lds {lds:6d} "
                  f"scratch {priv:4d}{flag}", flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
