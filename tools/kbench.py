"""Kernel A/B timing on the bench panel: python tools/kbench.py [lib.so ...]
Each library (default: the in-tree one) runs in its own subprocess (FM_HIP_LIB); one
pipeline pass fills engine.LAST_LAUNCH, then every tag's latest launch is re-issued back to
back (engine.time_launch) several times; the median per tag is printed."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    sys.path[:0] = [os.path.join(ROOT, "fm-returnprediction_amd"), ROOT]
    import numpy as np
    import torch
    from fmcore import engine as E
    from fmcore import lewellen as LW
    dev = E.require_device()
    # KB_PLANES=2: the planes-only panel bench.py times (fm_gen_panel_planes, no FP64 columns)
    panel = E.panel_synthetic(600, 5000, 1, device=dev, layout="planes" if os.environ.get("KB_PLANES") == "2" else "f64")
    if os.environ.get("KB_CHUNK"):   # Gram chunk-size A/B (rows per workgroup)
        panel.chunk_rows = int(os.environ["KB_CHUNK"])
    pol = os.environ.get("KB_POLICY", "")
    if pol == "months":   # whole-month Gram chunks instead of the default plan
        panel.chunk_policy = ("months", panel.max_seg_len)
    if os.environ.get("KB_SLOTS"):   # the balanced plan cut for this many workgroups
        panel.chunk_policy = E.chunk_policy(panel.nrows, panel.nseg, panel.max_seg_len, slots=int(os.environ["KB_SLOTS"]))

    if os.environ.get("KB_PLANES") == "1":   # FP64 columns + the split planes (fm_split_planes)
        E.split_planes(panel)
    cfg = LW.PipelineConfig()
    for _ in range(3):
        LW.run_pipeline(panel, cfg)
    torch.cuda.synchronize()
    out = {}
    for tag in sorted(E.LAST_LAUNCH):
        ts = [E.time_launch(tag, 10) for _ in range(7)]
        out[tag] = float(np.median(ts))
    print("KB " + json.dumps(out))


def main():
    if os.environ.get("KB_CHILD") == "1":
        return child()
    libs = sys.argv[1:] or [os.path.join(ROOT, "fm-returnprediction_amd", "lib", "libfm_hip.so")]
    for lib in libs:
        env = dict(os.environ, KB_CHILD="1", FM_HIP_LIB=os.path.abspath(lib))
        r = subprocess.run([sys.executable, __file__], env=env, capture_output=True, text=True, timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith("KB ")]
        if not line:
            print(lib, "FAILED", r.stderr[-2000:])
            continue
        d = json.loads(line[0][3:])
        tag = os.path.basename(os.path.dirname(lib)) + (f"[chunk {os.environ['KB_CHUNK']}]" if os.environ.get("KB_CHUNK") else "")
        tag += "".join(f"[{k}={os.environ[k]}]" for k in ("KB_POLICY", "KB_PLANES", "KB_SLOTS") if os.environ.get(k))
        print(tag, " ".join(f"{k}={v * 1e3:.1f}us" for k, v in d.items()), flush=True)


if __name__ == "__main__":
    main()
