"""Summarise lab_pipe_prof output: per-phase clock64 cycles (median / mean)."""
import sys
import numpy as np

a = np.fromfile(sys.argv[1], dtype=np.int64).reshape(-1, 16, 4, 4)  # block, step, wave, phase
wall = a[:, 15, :, :2].copy()  # wall_clock64 (100 MHz) start / end per wave
a = a[:, :15]
valid = a[..., 0] != 0
print("blocks", a.shape[0], "steps with data", valid.any(axis=2).sum(axis=1).mean())
comp = (a[..., 1] - a[..., 0])[valid]
bar1 = (a[..., 2] - a[..., 1])[valid]
stw = (a[..., 3] - a[..., 2])[valid]
# barrier 2 + loop top: next step's start - this step's phase 3
nxt = np.zeros_like(a[..., 0])
nxt[:, :-1] = a[:, 1:, :, 0] - a[:, :-1, :, 3]
v2 = valid.copy(); v2[:, -1] = False; v2 &= np.concatenate([valid[:, 1:], np.zeros_like(valid[:, :1])], axis=1)
bar2 = nxt[v2]
for name, x in (("compute", comp), ("barrier1 wait", bar1), ("staging write (incl vmcnt wait)", stw), ("barrier2+top", bar2)):
    print(f"{name:34s} median {np.median(x):8.0f}  mean {x.mean():8.0f}  p90 {np.percentile(x, 90):8.0f}")
ws = wall[:, 0, 0]; we = wall[:, :, 1].max(axis=1)
ok = ws > 0
w0 = ws[ok].min()
print("wall (us): block start median %.2f p90 %.2f max %.2f | end median %.2f p90 %.2f max %.2f | dur median %.2f max %.2f" % (
    np.median(ws[ok] - w0) / 100, np.percentile(ws[ok] - w0, 90) / 100, (ws[ok] - w0).max() / 100,
    np.median(we[ok] - w0) / 100, np.percentile(we[ok] - w0, 90) / 100, (we[ok] - w0).max() / 100,
    np.median(we[ok] - ws[ok]) / 100, (we[ok] - ws[ok]).max() / 100))
steps = valid.any(axis=2).sum(axis=1)
for k in sorted(set(steps.tolist())):
    sel = ok & (steps == k)
    if sel.any():
        print(f"  blocks with {k} steps: {sel.sum():4d}  dur median {np.median(we[sel] - ws[sel]) / 100:.2f} us")
t0 = a[..., 0][valid].min()
tend = a[..., 3][valid].max()
xcd = np.arange(a.shape[0]) & 7
for x in range(8):
    sel = ok & (xcd == x)
    d = (we[sel] - ws[sel]) / 100
    c = (a[..., 1] - a[..., 0])[sel][valid[sel]]
    print(f"  XCD {x}: blocks {sel.sum():3d} dur median {np.median(d):.2f} max {d.max():.2f} us; steps mean {steps[sel].mean():.2f}; compute/step median {np.median(c):.0f}")
