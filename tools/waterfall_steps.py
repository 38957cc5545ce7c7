#!/usr/bin/env python3
# Per-kernel durations of the waterfall steps in a one-stream rocprofv3 kernel trace of the default bench:
#   python3 tools/waterfall_steps.py <run_kernel_trace.csv>   (a step starts at its ofdm_rx launch; waterfall steps
#   are those whose first gather takes > 0.1 ms; the first two are skipped as warm-up)
import csv,sys,collections
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
def short(n):
    for k in ('tdec_kernel_p2x','tdec_kernel_p2c','tdec_kernel_p2s','tdec_cont_gather2','tdec_cont_gather','tdec_cont_assign2','tdec_cont_assign','rm_combine','rm_direct_map','ofdm_rx','chest','tb_kernel'):
        if k in n: return k
    return n[:30]
# split into steps at each p2x launch
steps=[]; cur=None
for r in rows:
    k=short(r['Kernel_Name']); d=(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e6
    if k=='ofdm_rx': cur=[]; steps.append(cur)
    if cur is not None: cur.append((k,d,int(r['Start_Timestamp']),int(r['End_Timestamp'])))
wf=[s for s in steps if any(k=='tdec_cont_gather' and d>0.1 for k,d,_,_ in s)]
print('steps',len(steps),'waterfall steps',len(wf))
agg=collections.defaultdict(list)
for s in wf[2:]:
    seen=collections.Counter()
    for k,d,_,_ in s:
        seen[k]+=1
        agg[(k,seen[k])].append(d)
    agg[('wall',1)].append((s[-1][3]-s[0][2])/1e6)
for (k,i),v in sorted(agg.items(), key=lambda x: (x[0][0]!='wall', x[0][0], x[0][1])):
    print('%-22s #%d  n=%3d  avg %.3f ms'%(k,i,len(v),sum(v)/len(v)))
