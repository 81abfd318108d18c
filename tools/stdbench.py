"""calc_std_12 rolling-std timing: python tools/stdbench.py [lib.so ...]
5,000 firms x 2,520 trading days of synthetic daily returns in HBM (bench.py firm_chars'
panel); fm_rolling_std (252-day window, min 100) timed with HIP events over 20 launches,
each library in its own subprocess (FM_HIP_LIB).  Prints ms per launch and GB/s of the
24 algorithmic bytes per row."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    sys.path[:0] = [os.path.join(ROOT, "fm-returnprediction_amd"), ROOT]
    import torch
    from fmcore import engine as E
    from fmcore import synth_chars
    E.require_device()
    dids, x = synth_chars.device_daily_returns(5000, 2520, seed=1)
    out = torch.empty_like(x)
    for _ in range(3):
        E.rolling_std(dids, x, out=out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        E.rolling_std(dids, x, out=out)
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / 20
    print("SB " + json.dumps({"ms": ms, "rows": int(x.shape[0])}))


def main():
    if os.environ.get("SB_CHILD") == "1":
        return child()
    libs = sys.argv[1:] or [os.path.join(ROOT, "fm-returnprediction_amd", "lib", "libfm_hip.so")]
    for lib in libs:
        env = dict(os.environ, SB_CHILD="1", FM_HIP_LIB=os.path.abspath(lib))
        r = subprocess.run([sys.executable, __file__], env=env, capture_output=True, text=True, timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith("SB ")]
        if not line:
            print(lib, "FAILED", r.stderr[-2000:])
            continue
        d = json.loads(line[0][3:])
        tag = os.path.basename(os.path.dirname(lib))
        print(f"{tag}: {d['ms']:.4f} ms  {d['rows'] * 24 / (d['ms'] * 1e-3) / 1e9:.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
