"""Synthetic raw CRSP/Compustat inputs for the firm-axis characteristic kernels (bench and
full-size parity tests).  Generated on the device with a seeded torch generator (data only:
no product arithmetic happens here).

Layout is the one fm_firm_chars / fm_rolling_std take: FIRM-major, each firm's rows
contiguous in date order — what get_factors produces with
sort_values(["permno", "mthcaldt"]) (reference src/calc_Lewellen_2014.py:533).
"""
from __future__ import annotations

import torch

from .engine import CHAR_FIELDS


def device_raw_panel(nfirms: int, nmonths: int, seed: int = 0, nan_rate: float = 0.02, device="cuda"):
    """Balanced firm-major monthly panel: ids int64 [F*T], fields {name: float64 [F*T]}."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    n = nfirms * nmonths
    ids = (torch.arange(nfirms, dtype=torch.int64, device=device) + 10000).repeat_interleave(nmonths)

    def normal(mu, sd):
        return torch.randn(n, generator=g, dtype=torch.float64, device=device) * sd + mu

    f = {}
    f["me"] = torch.exp(normal(5.0, 2.0))
    f["be"] = f["me"] * torch.exp(normal(-0.5, 0.8))
    f["retx"] = normal(0.01, 0.1).clamp_min(-0.95)
    f["accruals"] = normal(0.0, 0.05)
    f["depreciation"] = normal(0.03, 0.01).abs()
    f["earnings"] = normal(2.0, 10.0)
    f["assets"] = torch.exp(normal(6.0, 1.5))
    f["dvc"] = torch.where(torch.rand(n, generator=g, device=device, dtype=torch.float64) < 0.7,
                           torch.zeros(n, dtype=torch.float64, device=device), normal(0.5, 0.3).abs())
    f["prc"] = torch.exp(normal(3.0, 1.0))
    f["shrout"] = torch.exp(normal(9.0, 1.0))
    f["total_debt"] = normal(100.0, 60.0).abs()
    f["sales"] = normal(300.0, 200.0).abs()
    for k in CHAR_FIELDS:
        miss = torch.rand(n, generator=g, device=device, dtype=torch.float64) < nan_rate
        f[k] = torch.where(miss, torch.full_like(f[k], float("nan")), f[k])
    return ids, f


def device_daily_returns(nfirms: int, ndays: int, seed: int = 0, nan_rate: float = 0.02, device="cuda"):
    """Balanced firm-major daily returns: ids int64 [F*D], retx float64 [F*D]."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    n = nfirms * ndays
    ids = (torch.arange(nfirms, dtype=torch.int64, device=device) + 10000).repeat_interleave(ndays)
    x = torch.randn(n, generator=g, dtype=torch.float64, device=device) * 0.02 + 0.0005
    miss = torch.rand(n, generator=g, device=device, dtype=torch.float64) < nan_rate
    x = torch.where(miss, torch.full_like(x, float("nan")), x)
    return ids, x
