"""Summarise rocprofv3 PMC CSVs per kernel (mean per dispatch)."""
import csv, glob, sys, collections
root = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(root + '/**/*counter_collection.csv', recursive=True):
  per = collections.defaultdict(float)
  names = {}
  for r in csv.DictReader(open(f)):
    k = (r['Dispatch_Id'], r['Counter_Name'])
    per[k] += float(r['Counter_Value'])
    names[r['Dispatch_Id']] = r['Kernel_Name']
  for (d, c), v in per.items():
    agg[names[d][:60]][c].append(v)
for kn, cs in agg.items():
  if 'lddl' not in kn: continue
  print(kn)
  for c, vs in sorted(cs.items()):
    print('   %-24s %.4g' % (c, sum(vs) / len(vs)))
for f in glob.glob(root + '/**/*kernel_stats.csv', recursive=True):
  for r in csv.DictReader(open(f)):
    if 'lddl' in r['Name']:
      print('%-60s calls %s avg %.3f ms' % (r['Name'][:60], r['Calls'], float(r['AverageNs']) / 1e6))
