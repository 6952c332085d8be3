#!/usr/bin/env python3
"""Per-kernel averages of the C3 profile and the C3 line (gpurun_out/prof_c3)."""
import csv, json
for r in csv.DictReader(open('gpurun_out/prof_c3/trace/run_kernel_stats.csv')):
    print("%-60s %6s %10.1f us %6s%%" % (r['Name'][:60], r['Calls'], float(r['AverageNs']) / 1e3, r['Percentage'][:5]))
d = json.loads(open('gpurun_out/prof_c3/c3.jsonl').read().strip().split('\n')[-1])
print("C3 value %.4g wall %.4f runs %s |dlogZ| %.4f sigma %.4f" % (d['value'], d['wall_s'], [round(x, 4) for x in d['wall_s_runs']],
      d['log_evidence']['abs_delta'], d['log_evidence']['sigma_H']))
