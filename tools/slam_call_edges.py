"""Kernels around one steady-state mapping(15) call in a prof_slam.sh trace: the launches right
before its first gather and right after its last Adam step (the call's setup and teardown)."""
import csv
import glob

f = glob.glob("/tmp/profs/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
adam = [i for i, e in enumerate(ev) if "k_adam_train" in e[2] or "k_adam_step_segments" in e[2]]
# the calls: runs of Adam launches no more than 40 kernels apart
calls, cur = [], [adam[0]]
for i in adam[1:]:
    if i - cur[-1] > 40:
        calls.append(cur)
        cur = [i]
    else:
        cur.append(i)
calls.append(cur)
call = calls[-3]
first = call[0]
while "k_train_gather" not in ev[first][2]:
    first -= 1
print(f"{len(calls)} calls; this one: {len(call)} iterations, kernels {first}..{call[-1]}, "
      f"span {(ev[call[-1]][1] - ev[first][0]) / 1e3:.1f} us")
for s, e, n in ev[first - 14:first]:
    print(f"  before {n.replace('(anonymous namespace)::', '')[:70]:70s} {(e - s) / 1e3:7.2f} us  ends {(ev[first][0] - e) / 1e3:8.2f} us before")
for s, e, n in ev[call[-1] + 1:call[-1] + 10]:
    print(f"  after  {n.replace('(anonymous namespace)::', '')[:70]:70s} {(e - s) / 1e3:7.2f} us  starts {(s - ev[call[-1]][1]) / 1e3:8.2f} us after")

# the frame's work before the call (process_frame and the grid rebuild): every kernel in the
# 1.6 ms before the call's first gather, with its start relative to that gather
t_first = ev[first][0]
print("kernels in the 1.6 ms before the call (start relative to its first gather, duration):")
for s, e, n in ev:
    if t_first - 1.6e6 <= s < t_first:
        print(f"  {(s - t_first) / 1e3:9.1f} us  {(e - s) / 1e3:7.2f} us  {n.replace('(anonymous namespace)::', '')[:80]}")
