"""Per-kernel hardware-counter summary of rocprofv3 ``--pmc`` passes (``--output-format csv``).

``python scripts/pmc_summary.py <pass_dir> [<pass_dir> ...] [--top N]`` merges the
``*_counter_collection.csv`` of several passes (one counter group per pass), groups dispatches by
kernel name and prints, per kernel: dispatches, mean duration, and the derived rates that exist for
the collected counters --
  * HBM traffic: FETCH_SIZE + WRITE_SIZE (KiB per dispatch) -> GB moved and achieved TB/s;
  * MFMA issue: SQ_INSTS_MFMA per dispatch -> matrix TFLOP/s actually executed, taking 32x32x16 bf16
    (32768 FLOP per wave instruction) for the attention kernels and 16x16x32 bf16 (16384) for the GEMMs
    (ours: gemm.hip / skinny.hip; hipBLASLt: the ``MI16x16`` in the kernel name);
  * SQ_INSTS_VALU / SQ_INSTS_MFMA (VALU work per matrix instruction), LDS bank conflicts.
Durations come from the Start/End timestamps of each dispatch record.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace("void ", "")
    for pre in ("dalle::", "_ZN5dalle"):
        if name.startswith(pre):
            break
    return name[:70]


def main(argv):
    top = 25
    if "--top" in argv:
        i = argv.index("--top")
        top = int(argv[i + 1])
        del argv[i:i + 2]
    per = defaultdict(lambda: defaultdict(float))       # kernel -> counter -> sum over dispatches
    durs = defaultdict(dict)                            # kernel -> {(pass, dispatch): ns}
    for pi, d in enumerate(argv):
        for path in glob.glob(os.path.join(d, "*counter_collection.csv")):
            for r in csv.DictReader(open(path)):
                k = short(r["Kernel_Name"])
                per[k][r["Counter_Name"]] += float(r["Counter_Value"])
                durs[k][(pi, r["Dispatch_Id"])] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    rows = []
    for k, c in per.items():
        n = len({dk for dk in durs[k]})
        npass = max(1, len({p for p, _ in durs[k]}))
        disp = n / npass
        t_ns = sum(durs[k].values()) / max(1, n)
        rows.append((t_ns * disp, k, disp, t_ns, c))
    rows.sort(reverse=True)
    print(f"{'kernel':70} {'disp':>5} {'avg_us':>8} {'GB/disp':>8} {'TB/s':>6} {'MFMA/disp':>10} {'MFMA_TF/s':>9} {'valu/mfma':>9} {'lds_conf':>9}")
    for _, k, disp, t_ns, c in rows[:top]:
        def avg(name):
            return c[name] / disp if name in c else None
        fetch, write = avg("FETCH_SIZE"), avg("WRITE_SIZE")
        gb = ((fetch or 0) + (write or 0)) * 1024 / 1e9 if (fetch is not None or write is not None) else None
        tbs = gb / (t_ns * 1e-9) / 1e3 if gb is not None and t_ns > 0 else None
        mf = avg("SQ_INSTS_MFMA")
        fpi = 32768.0 if "attn" in k else 16384.0
        busy = mf * fpi / (t_ns * 1e-9) / 1e12 if mf and t_ns > 0 else None
        vpm = (c["SQ_INSTS_VALU"] / c["SQ_INSTS_MFMA"]) if c.get("SQ_INSTS_MFMA") and "SQ_INSTS_VALU" in c else None
        lds = avg("SQ_LDS_BANK_CONFLICT")
        fmt = lambda v, f: (f % v) if v is not None else "-"  # noqa: E731
        print(f"{k:70} {disp:5.0f} {t_ns / 1e3:8.1f} {fmt(gb, '%8.3f'):>8} {fmt(tbs, '%6.2f'):>6} {fmt(mf, '%10.3g'):>10} "
              f"{fmt(busy, '%9.1f'):>9} {fmt(vpm, '%9.1f'):>9} {fmt(lds, '%9.3g'):>9}")


if __name__ == "__main__":
    main(sys.argv[1:])
