"""C5-shaped select timing: python tools/selbench.py [lib.so ...]
A 1,000-month x 20,000-firm x 15-column synthetic panel (fm_gen_panel) in HBM; fm_select_cuts
(1/99 cuts + Gram pivot, as local_stage calls it) timed with HIP events over 5 launches,
each library in its own subprocess (FM_HIP_LIB).  Prints ms per launch and GB/s of the
columns read once."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    sys.path[:0] = [os.path.join(ROOT, "fm-returnprediction_amd"), ROOT]
    import torch
    from fmcore import engine as E
    E.require_device()
    T, N = int(os.environ.get("SB_T", "1000")), int(os.environ.get("SB_N", "20000"))
    p = E.panel_synthetic(T, N, 20150101, month0=50000)
    if os.environ.get("SB_PLANES", "1") == "1":   # the bench's split panel (high-plane selects)
        E.split_planes(p)
    for _ in range(2):
        E.select_cuts(p, 0.01, 0.99, 5, center=True)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        E.select_cuts(p, 0.01, 0.99, 5, center=True)
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / 5
    gbs = T * N * p.ncols * 8 / (ms * 1e-3) / 1e9
    print("SB " + json.dumps({"ms": ms, "gbs": gbs, "T": T, "N": N}))


def main():
    if os.environ.get("SB_CHILD") == "1":
        return child()
    libs = sys.argv[1:] or [os.path.join(ROOT, "fm-returnprediction_amd", "lib", "libfm_hip.so")]
    for lib in libs:
        env = dict(os.environ, SB_CHILD="1", FM_HIP_LIB=os.path.abspath(lib))
        r = subprocess.run([sys.executable, __file__], env=env, capture_output=True, text=True, timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith("SB ")]
        tag = os.path.basename(os.path.dirname(lib))
        if not line:
            print(tag, "FAILED", r.stderr[-2000:], flush=True)
            continue
        d = json.loads(line[0][3:])
        print(f"{tag}: {d['ms']:.3f} ms  {d['gbs']:.0f} GB/s  ({d['T']}x{d['N']})", flush=True)


if __name__ == "__main__":
    main()
