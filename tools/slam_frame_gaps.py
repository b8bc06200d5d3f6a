"""Where the GPU waits inside a SLAM frame: from a prof_slam.sh kernel trace (/tmp/profs), the
span between the ends of consecutive mapping calls (one frame), the kernels' busy time inside it,
and every idle gap longer than GAP us with the kernels on either side -- the host-bound stretches
(count reads, Python between launches)."""
import csv
import glob
import os

GAP = float(os.environ.get("GAP", "4"))
f = glob.glob("/tmp/profs/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
name = lambda s: s.replace("(anonymous namespace)::", "").replace("void ", "")[:58]  # noqa: E731
adam = [i for i, e in enumerate(ev) if "k_adam_train" in e[2]]
ends, cur = [], [adam[0]]
for i in adam[1:]:
    if i - cur[-1] > 40:
        ends.append(cur[-1])
        cur = [i]
    else:
        cur.append(i)
ends.append(cur[-1])
print(f"{len(ends)} mapping calls")
for a, b in zip(ends[-4:-1], ends[-3:]):
    span = ev[b][1] - ev[a][1]
    busy, gaps, t = 0, [], ev[a][1]
    for j in range(a + 1, b + 1):
        s, e, n = ev[j]
        if s - t > GAP * 1e3:
            gaps.append(((s - t) / 1e3, name(ev[j - 1][2]), name(n)))
        busy += max(0, e - max(s, t))
        t = max(t, e)
    print(f"\nframe: span {span / 1e3:.1f} us, kernels busy {busy / 1e3:.1f} us, idle {(span - busy) / 1e3:.1f} us, "
          f"{b - a} kernels; gaps > {GAP} us:")
    for g, p, n in gaps:
        print(f"  {g:8.1f} us  after {p:58s} before {n}")

if os.environ.get("FULL"):
    a, b = ends[-3], ends[-2]
    print("\nfull sequence of the last frame (gap before each kernel, us; duration, us):")
    t = ev[a][1]
    for j in range(a + 1, b + 1):
        s, e, n = ev[j]
        print(f"  {(s - t) / 1e3:8.1f}  {(e - s) / 1e3:7.1f}  {name(n)}")
        t = max(t, e)
