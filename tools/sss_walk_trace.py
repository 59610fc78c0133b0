"""Per-iteration GPU timeline of SSS walks from a rocprofv3 kernel_trace.csv:
mean k_sss_eval / k_sss_post durations, the gap from an eval's end to its
post's start and from a post's end to the next eval's start (the host's share
of the critical path when the GPU is idle), over the walks' steady iterations.
usage: python tools/sss_walk_trace.py run_kernel_trace.csv [...]"""
import csv
import statistics as st
import sys

for path in sys.argv[1:]:
    rows = list(csv.DictReader(open(path)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows
                if "k_sss_eval" in r["Kernel_Name"] or "k_sss_post" in r["Kernel_Name"])
    ev, po, g_ep, g_pe = [], [], [], []
    for i in range(len(ks) - 2):
        a, b, c = ks[i], ks[i + 1], ks[i + 2]
        if "k_sss_eval" in a[2] and "k_sss_post" in b[2]:
            ev.append((a[1] - a[0]) / 1e3)
            po.append((b[1] - b[0]) / 1e3)
            g_ep.append((b[0] - a[1]) / 1e3)
            if "k_sss_eval" in c[2] and (c[0] - b[1]) < 100e3:  # same walk
                g_pe.append((c[0] - b[1]) / 1e3)
    med = lambda x: st.median(x) if x else float("nan")  # noqa: E731
    print(f"{path}: {len(ev)} iterations; median us: eval {med(ev):.1f}, post {med(po):.1f}, "
          f"eval->post gap {med(g_ep):.1f}, post->next eval gap {med(g_pe):.1f}; "
          f"iteration span {med(ev) + med(po) + med(g_ep) + med(g_pe):.1f}")
