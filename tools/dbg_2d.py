import sys, numpy as np, torch
sys.path.insert(0, '.')
from crimp_amd import ops, _native as N
from crimp_amd.synth import pulsed_events
dev = torch.device("cuda", 0)
t_h = pulsed_events(200_000, 2.0e5, 7.123456789, pulsed_frac=0.05, seed=11)
f_h = 7.123456789 + (np.arange(40_000) - 20_000) / 2.0e6
fd = np.array([-12.0, -10.5])
t = torch.as_tensor(t_h, device=dev); f = torch.as_tensor(f_h, device=dev); fdd = torch.as_tensor(fd, device=dev)
t0 = float((t[0] + t[-1]).item()) / 2
L = N.load()
full = ops.search(t, t0, f, 2, 0, log10_negfdot=fdd).cpu().numpy(); nfx = L.crimp_last_fixups()
full2 = ops.search(t, t0, f, 2, 0, log10_negfdot=fdd).cpu().numpy()
a = ops.search(t, t0, f, 2, 0, log10_negfdot=fdd, first=0, count=40000).cpu().numpy(); na = L.crimp_last_fixups()
b = ops.search(t, t0, f, 2, 0, log10_negfdot=fdd, first=40000, count=40000).cpu().numpy(); nb = L.crimp_last_fixups()
print("repeat equal", np.array_equal(full, full2), "fixups", nfx, na, nb)
for nm, x, ref in (("row0", a, full[:40000]), ("row1", b, full[40000:])):
    bad = np.nonzero(x != ref)[0]
    print(nm, "mismatch", bad.size, bad[:8], "rel", (np.abs(x - ref) / np.abs(ref))[bad[:5]] if bad.size else "")
    if bad.size: print("   tiles", np.unique(bad // 1024)[:20], "pos hist", np.bincount((bad % 1024) // 128, minlength=8))
th = t_h; fh = f_h
a2 = ops.search(th, t0, fh, 2, 0, log10_negfdot=fd, first=0, count=40000)
print("host row0 == device row0", np.array_equal(a2, a))
