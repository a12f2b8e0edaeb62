"""Is a short train_steps call slower per step than a long one, and where?
B = 20 (configs[1]), graphs prepared.  Run mode (no profiler): wall time per
call for calls of n = 20 and 200 steps, each after a synchronize.  Under
rocprofv3 --kernel-trace (mode "trace"): the same calls, then
    python tools/steps_warm.py analyze <run_kernel_trace.csv>
prints the span of each step (first kernel start -> next step's first kernel
start) by its index inside the 20-step calls, against the 200-step call's.
    python tools/steps_warm.py run|trace|first"""
import csv
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
FIRST = "smallm_kernel<false, 2, 1>"   # a step's first launch (the input Dense, 52 workgroups)


def analyze(path):
    rows = []
    for r in csv.DictReader(open(path)):
        gx = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0)
        wx = int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", 1)) or 1)
        rows.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), gx // max(wx, 1)))
    rows.sort(key=lambda r: r[1])
    starts = [s for n, s, e, wg in rows if FIRST in n and wg == 52]
    ends = [e for n, s, e, wg in rows]
    # calls: runs of steps separated by > 30 us of idle before a step's first kernel
    calls, cur = [], []
    last_end = {s: max(e for _, s2, e, _ in rows if s2 < s) if any(s2 < s for _, s2, _, _ in rows) else s
                for s in starts}
    for s in starts:
        if cur and s - last_end[s] > 30_000:
            calls.append(cur)
            cur = []
        cur.append(s)
    if cur:
        calls.append(cur)
    end_all = max(ends)
    for ci, c in enumerate(calls):
        # span of step j: its start to the next step's start (the last: to the last kernel end before the next call)
        nxt = calls[ci + 1][0] if ci + 1 < len(calls) else end_all + 1
        last = max(e for _, s, e, _ in rows if c[-1] <= s < nxt)
        spans = [(c[j + 1] - c[j]) / 1e3 for j in range(len(c) - 1)] + [(last - c[-1]) / 1e3]
        head = " ".join(f"{v:6.1f}" for v in spans[:6])
        print(f"call {ci:2d}: {len(c):4d} steps, span {sum(spans):8.1f} us, mean {sum(spans) / len(spans):6.2f}, "
              f"first 6 steps [{head}], mean of steps 10+ {sum(spans[10:]) / max(1, len(spans[10:])):6.2f}")


def main():
    mode = sys.argv[1]
    if mode == "analyze":
        return analyze(sys.argv[2])
    import torch
    import bench
    from iwae_replication_project_amd import Adam, Flexible_Model

    B = bench.B_PER_GPU
    x, pi = bench.synthetic_images(400 * B, 1)
    m = Flexible_Model(bench.HE, bench.HD, bench.LE, bench.LD, dataset_bias=pi, loss_function="IWAE", k=bench.K,
                       seed=2)
    m.compile(Adam(learning_rate=1e-3, epsilon=1e-4))
    xd = m._x(x)
    for n in (20, 200):
        m.prepare_train_steps(xd[:n * B], B)
    if mode == "first":
        m.prepare_train_steps(xd[:200 * B], B)
    m.train_steps(xd[:200 * B], B, sync=False)
    torch.cuda.synchronize()
    if mode == "first":
        # the first replay of a prepared (captured, uploaded, never launched)
        # 20-step graph against its later replays, GPU hot from a 200-step call;
        # then 20 steps as five 4-step graph launches back to back (one sync)
        for n in (4,):
            m.prepare_train_steps(xd[:n * B], B)
        w = []
        for _ in range(6):
            torch.cuda.synchronize()
            t = time.perf_counter()
            m.train_steps(xd[:20 * B], B, sync=False)
            m._stream.synchronize()
            w.append((time.perf_counter() - t) * 1e6)
        print("20-step graph, calls 1..6 (the first = its first replay), us/step:",
              " ".join(f"{v / 20:.2f}" for v in w), flush=True)
        m.train_steps(xd[:4 * B], B, sync=False)
        w = []
        for _ in range(6):
            torch.cuda.synchronize()
            t = time.perf_counter()
            for j in range(5):
                m.train_steps(xd[4 * j * B:4 * (j + 1) * B], B, sync=False)
            m._stream.synchronize()
            w.append((time.perf_counter() - t) * 1e6)
        print("20 steps as five 4-step graph launches, us/step:", " ".join(f"{v / 20:.2f}" for v in w), flush=True)
        return
    reps = 6 if mode == "trace" else 20
    for n in (20, 200, 20):
        w = []
        for _ in range(reps if n == 20 else 3):
            torch.cuda.synchronize()
            t = time.perf_counter()
            m.train_steps(xd[:n * B], B, sync=False)
            m._stream.synchronize()
            w.append((time.perf_counter() - t) * 1e6)
        w.sort()
        print(f"n {n:4d}: wall per call median {w[len(w) // 2]:9.1f} us = {w[len(w) // 2] / n:7.2f} us/step "
              f"(min {w[0] / n:7.2f})", flush=True)


if __name__ == "__main__":
    main()
