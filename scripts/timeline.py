#!/usr/bin/env python3
"""Step timeline of a rocprofv3 --kernel-trace CSV (bench.py run): steps are delimited by the launches of
k_copy_multi (preTimeStep, one per dfmi_time_step). For the steps given, prints the wall time of each step,
the time the GPU had at least one kernel running (union of kernel intervals), the idle gaps, the busy time
per HIP queue (compute stream / side stream) and the kernels that run while nothing else does.

  python scripts/timeline.py <kernel_trace.csv> [first_step last_step] [--json out.json]
"""
import collections
import csv
import json
import sys


def load(path):
    rows = []
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r.get("Queue_Id", "0")))
    rows.sort()
    return rows


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    gaps = []
    for s, e in sorted(iv):
        if cur_e is None:
            cur_s, cur_e = s, e
        elif s > cur_e:
            tot += cur_e - cur_s
            gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot, gaps


def main(argv):
    out = None
    if "--json" in argv:
        i = argv.index("--json"); out = argv[i + 1]; argv = argv[:i] + argv[i + 2:]
    rows = load(argv[0])
    starts = [r[0] for r in rows if r[2].endswith("k_copy_multi")]
    first, last = (int(argv[1]), int(argv[2])) if len(argv) >= 3 else (len(starts) // 2, len(starts) - 2)
    res = {"steps": []}
    per_kernel = collections.Counter()
    excl = collections.Counter()
    for s in range(first, last + 1):
        t0, t1 = starts[s], starts[s + 1]
        win = [r for r in rows if t0 <= r[0] < t1]
        busy, gaps = union([(r[0], min(r[1], t1)) for r in win])
        q = collections.defaultdict(list)
        for r in win:
            q[r[3]].append((r[0], r[1]))
            per_kernel[r[2]] += r[1] - r[0]
        # time during which exactly one kernel runs, charged to it (the critical-path candidates)
        ev = sorted([(r[0], 1, i) for i, r in enumerate(win)] + [(r[1], -1, i) for i, r in enumerate(win)])
        running = set()
        last_t = t0
        for t, d, i in ev:
            if len(running) == 1:
                excl[win[next(iter(running))][2]] += t - last_t
            last_t = t
            if d > 0:
                running.add(i)
            else:
                running.discard(i)
        res["steps"].append({"step": s, "wall_us": (t1 - t0) / 1e3, "busy_us": busy / 1e3,
                             "idle_us": (t1 - t0 - busy) / 1e3, "gaps": len(gaps),
                             "gaps_over_5us": sum(1 for g in gaps if g > 5000),
                             "idle_in_gaps_over_5us": sum(g for g in gaps if g > 5000) / 1e3,
                             "queue_busy_us": {k: union(v)[0] / 1e3 for k, v in q.items()},
                             "launches": len(win)})
    n = last - first + 1
    res["kernel_us_per_step"] = {k: v / 1e3 / n for k, v in per_kernel.most_common(40)}
    res["alone_us_per_step"] = {k: v / 1e3 / n for k, v in excl.most_common(40)}
    for st in res["steps"]:
        print(f"step {st['step']}: wall {st['wall_us']:.0f} us, busy {st['busy_us']:.0f}, idle {st['idle_us']:.0f} "
              f"({st['gaps']} gaps, {st['gaps_over_5us']} > 5 us holding {st['idle_in_gaps_over_5us']:.0f} us), "
              f"queues {{{', '.join(f'{k}: {v:.0f}' for k, v in st['queue_busy_us'].items())}}}, {st['launches']} launches")
    print("kernel time per step (us), top 25:")
    for k, v in list(res["kernel_us_per_step"].items())[:25]:
        print(f"  {v:9.1f}  alone {res['alone_us_per_step'].get(k, 0.0):9.1f}  {k}")
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1:])
