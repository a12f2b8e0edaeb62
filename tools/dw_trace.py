"""Per-workgroup k-step timeline of the large-batch weight-gradient kernel
(dw_kernel) from a -DIWAE_DW_TRACE build (tools/build_debug.sh), run with
IWAE_HIP_LIB pointing at it: B=512 train steps with dw_wide=1, then per
workgroup its item, k steps, duration and the average split of a k step
(multiply issue / staging + next request / barrier wait), wall_clock64 ticks
of 10 ns.   python tools/dw_trace.py [alpha]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
from iwae_replication_project_amd import Adam, Flexible_Model  # noqa: E402

alpha = int(sys.argv[1]) if len(sys.argv) > 1 else 150
B = 512
x, pi = bench.synthetic_images(2 * B, 1)
m = Flexible_Model(bench.HE, bench.HD, bench.LE, bench.LD, dataset_bias=pi, loss_function="IWAE", k=50, seed=2,
                   tuning={"dw_wide": 1, "dw_alpha": alpha} if len(sys.argv) > 1 else {"dw_wide": 1})
m.compile(Adam(learning_rate=1e-3, epsilon=1e-4))
xd = m._x(x)
for i in range(4):
    m.train_step(xd[(i % 2) * B:(i % 2 + 1) * B], sync=False)
torch.cuda.synchronize()
K = 3 + 3 * 80 + 1
buf = (ctypes.c_ulonglong * (256 * K))()
dump = m._lib.iwae_dw_trace_dump
dump.restype = ctypes.c_int
n = dump(buf, 256 * K)
rows = []
for b in range(256):
    r = buf[b * K:(b + 1) * K]
    item, nk, t0, t1 = r[0] & 0xFFFF, r[1], r[2], r[K - 1]
    if nk == 0 or t1 <= t0:
        continue
    ks = min(nk + (nk & 1), 80)
    mul = sum(r[3 + 3 * j] - (r[5 + 3 * (j - 1)] if j else t0) for j in range(ks)) / ks
    stg = sum(r[4 + 3 * j] - r[3 + 3 * j] for j in range(ks)) / ks
    bar = sum(r[5 + 3 * j] - r[4 + 3 * j] for j in range(ks)) / ks
    rows.append((t1 - t0, b, item, nk, mul, stg, bar))
rows.sort(reverse=True)
tmin = min(buf[b * K + 2] for b in range(256) if buf[b * K + 1])
print("ticks of 10 ns; per k step: multiply issue / staging + request / barrier wait")
for d, b, item, nk, mul, stg, bar in rows[:40]:
    print(f"wg {b:3d} item {item:3d} nk {nk:3d}  start {buf[b * K + 2] - tmin:6d}  dur {d:6d}  per-k {d / max(nk, 1):7.1f}"
          f"   mul {mul:6.1f} stage {stg:6.1f} barrier {bar:6.1f}")
print(f"... {len(rows)} workgroups; shortest {rows[-1][0]}")
# every workgroup, compact: duration (us), k steps, per-k (us) -- the balance of the cost model
import collections
d = sorted(((r[0] / 100.0, r[3], r[0] / 100.0 / max(r[3], 1)) for r in rows), reverse=True)
print("all workgroups (us, k steps, us per k step):")
print("  ".join(f"{a:.0f}/{b}/{c:.2f}" for a, b, c in d))
hist = collections.Counter(int(a // 10) * 10 for a, _, _ in d)
print("duration histogram (10 us bins):", dict(sorted(hist.items())))
print(f"mean {sum(a for a, _, _ in d) / len(d):.1f} us, max {d[0][0]:.1f} us")
# per job: block shape, items, k steps, duration, time per k step (the cost model's unit)
per = collections.defaultdict(list)
for b in range(256):
    r = buf[b * K:(b + 1) * K]
    if r[1] == 0 or r[K - 1] <= r[2]:
        continue
    w = r[0]
    per[((w >> 16) & 0xFF, (w >> 24) & 0xFF, (w >> 32) & 0xFF, (w >> 40) & 1)].append((r[1], (r[K - 1] - r[2]) / 100.0))
print("job mtb ntb wide | items  k steps  dur us (mean / max)  us per k step  tiles")
for (jb, mtb, ntb, wide), v in sorted(per.items()):
    nk = sum(a for a, _ in v) / len(v)
    du = [b for _, b in v]
    print(f"{jb:3d} {mtb:3d} {ntb:3d} {wide:4d} | {len(v):5d}  {nk:7.1f}  {sum(du) / len(du):7.1f} / {max(du):6.1f}"
          f"  {sum(b / a for a, b in v) / len(v):8.3f}  {mtb * ntb:5d}")
