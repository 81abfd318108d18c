"""Slab ordering probe (VERDICT r03 "one effective panel read per step"): the local pass
(universe -> winsorize cuts -> Gram -> solve) over the 600-month x 5,000-firm bench panel as
ONE graph, against the same pass over two 300-month halves back to back (each half's select
leaves ~181 MB in the 256 MiB Infinity Cache for its Gram to re-read).  Prints ms per replay.
python tools/slab_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "fm-returnprediction_amd"), ROOT]
import torch  # noqa: E402
from fmcore import engine as E, lewellen as LW  # noqa: E402


def graph_of(fn):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    return g


def time_graph(g, n=50):
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        g.replay()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / n


def main():
    E.require_device()
    cfg, mc = LW.PipelineConfig(), LW.table2_models()
    N = 5000
    full = E.panel_synthetic(600, N, 1)
    whole = E.default_chunk_rows(600 * N, 600, N)
    full.chunk_rows = whole
    res = {"full_600": time_graph(graph_of(lambda: LW.local_stage(full, cfg, mc)))}
    for tag, rows in (("halves_whole_month_chunks", whole), ("halves_default_chunks", None)):
        halves = [E.panel_synthetic(300, N, 1, month0=0), E.panel_synthetic(300, N, 1, month0=300)]
        for h in halves:
            h.chunk_rows = rows
        res[tag] = time_graph(graph_of(lambda: [LW.local_stage(h, cfg, mc) for h in halves]))
        del halves
    for k, v in res.items():
        print(f"{k}: {v:.4f} ms", flush=True)


if __name__ == "__main__":
    main()
