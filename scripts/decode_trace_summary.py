"""Summarise a rocprofv3 kernel trace of the decode loop (scripts/gpu_prof_decode_trace.sh): over the last N
complete steps (a step ends with the sampler kernel) print the wall time per step, the GPU-busy time (union of
kernel intervals), the summed kernel time (> busy when the two half-batch chains overlap), idle gaps, and
per-kernel counts / mean durations per step.

    python scripts/decode_trace_summary.py gpurun_out/prof_dec/run_kernel_trace.csv [--steps 16]"""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=16)
    ap.add_argument("--chains", type=int, default=1,
                    help="sampler kernels per image-position step (one per batch-slice chain that runs its own graph)")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    ends = [i for i, (_, _, n) in enumerate(rows) if "sample_kernel" in n]
    n_ends = a.steps * a.chains
    if len(ends) < n_ends + 1:
        print(f"only {len(ends)} sampler kernels")
        return
    i0, i1 = ends[-n_ends - 1] + 1, ends[-1]
    win = rows[i0:i1 + 1]
    t0, t1 = win[0][0], max(e for _, e, _ in win)
    wall = (t1 - t0) / 1e3 / a.steps
    busy, cur_s, cur_e = 0, None, None
    gaps = []
    pair_gap = defaultdict(list)   # (previous kernel, next kernel) -> idle gaps between them
    prev_name = None
    for s, e, n in win:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append(s - cur_e)
                pair_gap[(prev_name, n)].append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            if cur_e is not None:
                pair_gap[(prev_name, n)].append(0)
            cur_e = max(cur_e, e)
        prev_name = n
    busy += cur_e - cur_s
    ksum = sum(e - s for s, e, _ in win)
    print(f"# {a.steps} decode steps: wall {wall:.1f} us/step, GPU busy {busy / 1e3 / a.steps:.1f}, summed kernel time "
          f"{ksum / 1e3 / a.steps:.1f} (overlap factor {ksum / max(busy, 1):.2f}), kernels/step {len(win) / a.steps:.0f}")
    gaps.sort()
    if gaps:
        print(f"# idle gaps: {len(gaps) / a.steps:.0f} per step, total {sum(gaps) / 1e3 / a.steps:.1f} us/step, "
              f"median {gaps[len(gaps) // 2] / 1e3:.2f} us, p90 {gaps[int(len(gaps) * 0.9)] / 1e3:.2f} us")
    short = lambda n: n.split("(")[0].replace("void ", "")[-60:]  # noqa: E731
    print("# idle us/step  transitions/step  mean_gap_us  previous -> next kernel")
    for (pn, nn), g in sorted(pair_gap.items(), key=lambda kv: -sum(kv[1]))[:12]:
        print(f"{sum(g) / 1e3 / a.steps:9.1f} {len(g) / a.steps:8.1f} {sum(g) / len(g) / 1e3:8.2f}  {short(pn or '')} -> {short(nn)}")
    per = defaultdict(list)
    for s, e, n in win:
        per[n].append(e - s)
    print("# us/step  calls/step  mean_us  kernel")
    for n, d in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        print(f"{sum(d) / 1e3 / a.steps:9.1f} {len(d) / a.steps:8.1f} {sum(d) / len(d) / 1e3:8.2f}  {n[:110]}")


if __name__ == "__main__":
    main()
