"""Tie bench.py's cpu_baseline (the oracle port, kind "port") to the reference itself.

Run in THIS container only (the reference never travels to the GPU box), with the oracle
interpreter of SURVEY.md Appendix A:

    PYTHONDONTWRITEBYTECODE=1 /opt/conda/bin/python3.9 tools/ref_vs_port_timing.py [months] [firms]

Both legs run the bench's pass on the same synthetic panel (fmcore/synth.py, the generator
bench.py's device panel is bit-identical to), single-threaded BLAS, in the same interpreter:
  reference: winsorize(15 columns, 1/99) -> get_subsets -> build_table_2 (3 models x 3
             universes, NW(4), formatted table) -> create_figure_1 (Figure-1 OLS x 2
             universes + rolling 120/60), i.e. /root/reference/src/calc_Lewellen_2014.py
             :505-529, :44-112, :674-868, :871-926 through tests/golden/gen_goldens.py's
             loader (AST-extracted functions, regressions.py imported as is);
  port:      oracle/fm_oracle.py pipeline_arrays (the same pass plus the forecast and
             predictive-slope extensions, which the reference does not have).
Writes profiles/ref_vs_port.json: rows/s of each and ref_over_port = port / reference time.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests", "golden"), os.path.join(ROOT, "fm-returnprediction_amd"), ROOT]
os.environ.setdefault("OMP_NUM_THREADS", "1")
os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")
os.environ.setdefault("MKL_NUM_THREADS", "1")

import numpy as np  # noqa: E402

import gen_goldens as G  # noqa: E402  (reference loader + statsmodels/pandas shims)
from fmcore import synth  # noqa: E402
from oracle import fm_oracle as O  # noqa: E402


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 120
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 5000
    seed = 1                                           # bench.py's C3/C4 panel seed
    df = synth.synth_frame(T, N, seed)
    rows = len(df)
    ns = G.load_calc(G.RecordingPlt(), G.sm)
    vd = dict(G.cases.VARIABLES_DICT)
    t0 = time.perf_counter()
    w = ns["winsorize"](df, list(synth.WINSOR_VARS), 1, 99)
    t1 = time.perf_counter()
    subsets = ns["get_subsets"](w)
    t2 = time.perf_counter()
    ns["build_table_2"](subsets, vd)
    t3 = time.perf_counter()
    ns["create_figure_1"](subsets)
    t4 = time.perf_counter()
    ref_s = t4 - t0

    a = synth.synth_arrays(T, N, seed)
    seg = np.zeros(T + 1, dtype=np.int64)
    np.cumsum(np.bincount(a["month"], minlength=T), out=seg[1:])
    cols = {name: a[name] for name in synth.WINSOR_VARS}
    models = {k: ("retx", v, (0, 1, 2)) for k, v in G.cases.MODELS.items()}
    models["Figure 1"] = ("retx", ["log_bm", "return_12_2", "log_issues_36", "accruals_final",
                                   "log_assets_growth"], (0, 2))
    p0 = time.perf_counter()
    O.pipeline_arrays(cols, seg, a["me"], a["nyse"].astype(bool), models, None)
    port_s = time.perf_counter() - p0
    out = {
        "sample": f"{T} months x {N} firms (synth seed {seed}), {rows} rows, 1 BLAS thread",
        "interpreter": sys.version.split()[0], "numpy": np.__version__,
        "statsmodels": G.sm.__version__ if hasattr(G.sm, "__version__") else None,
        "reference_seconds": ref_s,
        "reference_stages_seconds": {"winsorize": t1 - t0, "get_subsets": t2 - t1,
                                     "build_table_2": t3 - t2, "create_figure_1": t4 - t3},
        "reference_rows_per_s": rows / ref_s,
        "port_seconds": port_s,
        "port_rows_per_s": rows / port_s,
        "ref_over_port": port_s / ref_s,
        "note": "ref_over_port < 1: the reference takes 1/ref_over_port times as long as the port "
                "on the same rows; multiply bench.py's cpu_baseline.value by it for the reference's rate",
    }
    path = os.path.join(ROOT, "profiles", "ref_vs_port.json")
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
