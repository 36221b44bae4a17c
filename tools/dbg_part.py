"""Determinism probe of the default search on one config-3-sized workload: two identical calls and a two-way
trial partition must give bit-identical statistics (exact integer sums). CRIMP_LIB selects a library build."""
import os, sys, numpy as np, torch
sys.path.insert(0, '/root/repo' if os.path.exists('/root/repo') else '.')
from crimp_amd import ops, _native as N
from crimp_amd.synth import pulsed_events
n, M, span, f0 = 10_000_000, 1_000_000, 1.0e6, 7.123456789
t_h = pulsed_events(n, span, f0, pulsed_frac=0.1, seed=0)
f_h = f0 + (np.arange(M) - M // 2) / (10.0 * span)
t = torch.as_tensor(t_h, device="cuda"); f = torch.as_tensor(f_h, device="cuda")
t0 = (t_h[0] + t_h[-1]) / 2
P = os.environ.get("PREC") or None
z1 = ops.search(t, t0, f, 2, 0, precision=P).cpu().numpy(); n1 = N.load().crimp_last_fixups()
z2 = ops.search(t, t0, f, 2, 0, precision=P).cpu().numpy(); n2 = N.load().crimp_last_fixups()
print("repeat identical:", np.array_equal(z1, z2), "fixups", n1, n2, flush=True)
rb = np.nonzero(z1 != z2)[0]
if rb.size:
    rr = np.abs(z1 - z2)[rb] / np.abs(z1[rb])
    print("  repeat diffs", rb.size, "rel quantiles", np.quantile(rr, [0, 0.5, 0.9, 1]),
          "abs max", np.abs(z1 - z2)[rb].max(), "rows hist", np.bincount((rb % 1024) // 32, minlength=32), flush=True)
cut = M // 2 + 123
a = ops.search(t, t0, f, 2, 0, first=0, count=cut, precision=P).cpu().numpy(); na = N.load().crimp_last_fixups()
b = ops.search(t, t0, f, 2, 0, first=cut, count=M - cut, precision=P).cpu().numpy(); nb = N.load().crimp_last_fixups()
ab = np.concatenate([a, b])
bad = np.nonzero(ab != z1)[0]
print("partition mismatches", bad.size, "fixups", na, nb, flush=True)
if bad.size:
    tiles = np.unique(bad // 1024)
    print("tiles", tiles[:20], tiles.size)
    print("first bad", bad[:10], "rel", (np.abs(ab - z1) / z1)[bad[:10]])
    print("in a:", np.sum(bad < cut), "in b:", np.sum(bad >= cut))
    # within-tile positions
    print("pos in tile hist", np.bincount((bad % 1024) // 128, minlength=8))
