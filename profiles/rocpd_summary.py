"""Summarise a rocprofv3 rocpd database (or kernel_stats.csv) into the
per-kernel table committed under profiles/:  name, calls, avg_ms, total_ms.

    python profiles/rocpd_summary.py gpurun_out/prof/run_results.db > profiles/<round>_<tag>.csv
"""
import sqlite3
import sys


def main(path):
    c = sqlite3.connect(path)
    q = ("select s.kernel_name, count(*), avg(d.end-d.start)/1e6, sum(d.end-d.start)/1e6, "
         "min(d.end-d.start)/1e6, max(d.end-d.start)/1e6 "
         "from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id=s.id "
         "group by s.kernel_name order by 4 desc")
    print("kernel,calls,avg_ms,total_ms,min_ms,max_ms")
    for name, n, avg, tot, mn, mx in c.execute(q):
        print("%s,%d,%.4f,%.4f,%.4f,%.4f" % (name.replace(",", ";"), n, avg, tot, mn, mx))


if __name__ == "__main__":
    main(sys.argv[1])
