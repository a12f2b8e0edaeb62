"""Where a replayed train step's wall time goes, from a rocprofv3 kernel trace
(results .db or kernel_trace .csv) of consecutive train steps: per step the
period (first kernel's start to the next step's first kernel's start), the sum
of kernel durations, the gaps inside the step and the gap to the next step.
    python tools/step_gaps.py <trace> [first_kernel_substring] [skip_steps]
Steps are delimited by the launches whose name contains first_kernel_substring
(default 'smallm_kernel<false>'); the first skip_steps (default 5) are dropped,
and so is any step whose period exceeds 3x the median (the bench's phase
boundaries)."""
import re
import statistics
import sys

sys.path.insert(0, __import__("os").path.dirname(__file__))
from step_timeline import load  # noqa: E402


def main():
    rows = load(sys.argv[1])
    first = sys.argv[2] if len(sys.argv) > 2 else "smallm_kernel<false>"
    skip = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    starts = [i for i, r in enumerate(rows) if first in r[0]]
    steps = []
    for a, b in zip(starts, starts[1:]):
        sel = rows[a:b]
        period = rows[b][1] - sel[0][1]
        busy = sum(e - s for _, s, e, _, _ in sel)
        inner = sum(max(0, sel[i + 1][1] - sel[i][2]) for i in range(len(sel) - 1))
        tail = rows[b][1] - sel[-1][2]
        steps.append((period, busy, inner, tail, len(sel)))
    steps = steps[skip:]
    if not steps:
        print("no steps found")
        return
    med = statistics.median(s[0] for s in steps)
    steps = [s for s in steps if s[0] <= 3 * med]
    n = len(steps)

    def avg(i):
        return sum(s[i] for s in steps) / n / 1000

    print(f"steps {n}  kernels/step {statistics.mode(s[4] for s in steps)}")
    print(f"period      {avg(0):8.2f} us  (median {med / 1000:.2f})")
    print(f"kernels     {avg(1):8.2f} us")
    print(f"gaps inside {avg(2):8.2f} us")
    print(f"gap between {avg(3):8.2f} us")
    names = {}
    a = starts[skip] if len(starts) > skip else starts[0]
    b = starts[skip + 1] if len(starts) > skip + 1 else len(rows)
    for name, s, e, gx, wx in rows[a:b]:
        names.setdefault(re.sub(r"\(.*", "", name)[:60] + f" wg {gx // max(wx, 1)}", []).append((e - s) / 1000)
    for k, v in names.items():
        print(f"  {sum(v):7.2f} us  {k}")


if __name__ == "__main__":
    main()
