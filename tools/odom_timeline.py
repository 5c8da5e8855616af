"""Per-frame device timeline of the odometry chain from a rocprofv3 kernel (+ memory copy) trace of
tools/odom_probe.py: frames are delimited by k_pack4 (the first kernel of a frame).  For every frame:
the wall span (pack4 to the next pack4), the device-busy union of all kernels and copies, and the idle
gaps; the average kernel sequence of the steady frames with each kernel's offset from the frame start,
its duration and the idle time before it (the host's share of the critical path).

    python tools/odom_timeline.py <rocprof dir> [prefix=run] [--skip 20]
"""
import csv
import os
import sys
from collections import defaultdict


def short(name):
    n = name.split("(")[0].replace("void ", "")
    for p in ("ddlo::", "rocprim::ROCPRIM_400200_NS::detail::"):
        n = n.replace(p, "")
    return n[:48]


def main():
    d = sys.argv[1]
    prefix = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else "run"
    skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 20
    ev = []
    kt = os.path.join(d, f"{prefix}_kernel_trace.csv")
    for r in csv.DictReader(open(kt)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r.get("Queue_Id", "?")))
    mt = os.path.join(d, f"{prefix}_memory_copy_trace.csv")
    if os.path.exists(mt):
        for r in csv.DictReader(open(mt)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy:" + r.get("Direction", "?"), "copy"))
    ev.sort()
    starts = [i for i, e in enumerate(ev) if e[2].startswith("k_pack4")]
    frames = []
    for a, b in zip(starts, starts[1:]):
        frames.append(ev[a:b] + [(ev[b][0], ev[b][0], "<next>", "")])
    frames = frames[skip:]
    print(f"{len(frames)} frames after skipping {skip}")
    walls, busys = [], []
    seq_stats = defaultdict(list)
    for f in frames:
        t0 = f[0][0]
        wall = f[-1][0] - t0
        # busy union
        busy, cur_s, cur_e = 0, None, None
        idle_before = []
        for s, e, n, q in f[:-1]:
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                    idle_before.append((n, s - cur_e))
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        if cur_e is not None:
            busy += cur_e - cur_s
        walls.append(wall)
        busys.append(busy)
        occ = defaultdict(int)
        for s, e, n, q in f[:-1]:
            k = (n, occ[n])
            occ[n] += 1
            seq_stats[k].append((s - t0, e - s))
        for n, g in idle_before:
            seq_stats[("idle before " + n, 0)].append((0, g))
    avg = lambda v: sum(v) / len(v) if v else 0.0
    print(f"wall per frame {avg(walls) / 1e3:.1f} us, device busy (union) {avg(busys) / 1e3:.1f} us, "
          f"idle {avg([w - b for w, b in zip(walls, busys)]) / 1e3:.1f} us")
    # the average sequence: kernels present in >= 80 % of frames, by mean offset
    rows = []
    idle = []
    for (n, i), v in seq_stats.items():
        if n.startswith("idle before "):
            idle.append((sum(g for _, g in v) / len(frames), n[12:], len(v)))
            continue
        if len(v) >= 0.8 * len(frames):
            rows.append((avg([o for o, _ in v]), n, i, avg([du for _, du in v]), len(v)))
    rows.sort()
    print("\n| offset us | kernel | # in frame | dur us | frames |\n|---:|---|---:|---:|---:|")
    for o, n, i, du, c in rows:
        print(f"| {o / 1e3:.1f} | {n} | {i} | {du / 1e3:.1f} | {c} |")
    idle.sort(reverse=True)
    print("\nidle device time per frame, by the kernel that ends it (top 15):")
    for g, n, c in idle[:15]:
        print(f"  {g / 1e3:7.1f} us  before {n}  ({c} gaps)")


if __name__ == "__main__":
    main()
