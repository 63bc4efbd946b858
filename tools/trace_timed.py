"""Per-dispatch durations of the hot kernels from a rocprofv3 kernel trace,
and their average over the bench's timed region.

usage: python tools/trace_timed.py profiles/r01_final/trace_kernel_trace.csv --warmup 2 --steps 10

bench.py's C2 run launches, per volume, one fingerprint pass (fp_kernel, plus
a tiny bounds-checked launch when the volume has edge strips) and one budgeted
SHA-256 slice; vs_cdc_wait adds one drain slice.  Order of sha_slice_kernel
dispatches: warmup volumes (W slices + 1 drain), timed volumes (K slices + 1
drain), the single-volume run (1 slice + 1 drain).
"""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--warmup", type=int, default=2)
ap.add_argument("--steps", type=int, default=10)
a = ap.parse_args()
rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))


def durs(name, min_ms=0.0):
    return [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows
            if name in r["Kernel_Name"].split("(")[0]
            and (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 >= min_ms]


def spans(name, min_ms=0.0):
    return [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
            if name in r["Kernel_Name"].split("(")[0]
            and (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 >= min_ms]


sha = durs("sha_slice_kernel")
timed = sha[a.warmup + 1: a.warmup + 1 + a.steps + 1]
print("sha_slice_kernel dispatches (ms):", [round(x, 2) for x in sha])
print(f"  timed region: {len(timed)} launches, total {sum(timed):.1f} ms, "
      f"avg {sum(timed) / len(timed):.2f} ms, per volume {sum(timed) / a.steps:.2f} ms")
fp = durs("fp_kernel", 1.0)
ft = fp[a.warmup: a.warmup + a.steps]
print("fp_kernel volume passes (ms):", [round(x, 2) for x in fp])
print(f"  timed region: {len(ft)} launches, avg {sum(ft) / len(ft):.2f} ms")
# the SHA-256 time of the timed region outside every fingerprint window (the
# line's "sha256" stage): slices dispatched while the persistent fingerprint
# grid holds the CUs wait inside their span without hashing
ss = spans("sha_slice_kernel")[a.warmup + 1: a.warmup + 1 + a.steps + 1]
fw = spans("fp_kernel", 1.0)[a.warmup: a.warmup + a.steps]
inside = sum(max(0, min(e, fe) - max(b, fb)) for b, e in ss for fb, fe in fw) / 1e6
total = sum(e - b for b, e in ss) / 1e6
print(f"  sha_slice_kernel outside the fingerprint windows: {total - inside:.1f} ms "
      f"({(total - inside) / a.steps:.2f} per volume), inside {inside:.1f} ms")
