"""Per-kernel stats (calls, total, average) from a rocprofv3 sqlite (.db) output -- the csv stats equivalent."""
import collections, glob, sqlite3, sys

f = glob.glob(sys.argv[1] + "/**/*.db", recursive=True)[0] if not sys.argv[1].endswith(".db") else sys.argv[1]
c = sqlite3.connect(f)
tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
ks = [t for t in tabs if t.startswith("rocpd_info_kernel_symbol")][0]
kd = [t for t in tabs if t.startswith("rocpd_kernel_dispatch")][0]
names = {r[0]: r[1] for r in c.execute(f"select id, kernel_name from {ks}")}
agg = collections.defaultdict(list)
for kid, s, e in c.execute(f"select kernel_id, start, end from {kd}"):
    agg[names[kid]].append(e - s)
tot = sum(sum(v) for v in agg.values())
print("Name,Calls,TotalDurationNs,AverageNs,Percentage")
for k, v in sorted(agg.items(), key=lambda x: -sum(x[1])):
    print(f'"{k}",{len(v)},{sum(v)},{sum(v)/len(v):.1f},{100*sum(v)/tot:.2f}')
