"""Per-step GPU busy time and idle gaps from a rocprofv3 kernel trace (step = fused AdamW end to AdamW end).

    python tools/trace_steps.py gpurun_out/prof8b/run_kernel_trace.csv
"""
import csv, sys
from collections import defaultdict
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
starts=[i for i,r in enumerate(rows) if 'rmsnorm_fwd' in r['Kernel_Name']]
# step boundary: adam kernel end
ad=[i for i,r in enumerate(rows) if 'adam_mt' in r['Kernel_Name']]
print('adam idx', ad)
for a,b in zip(ad[:-1], ad[1:]):
    seg=rows[a+1:b+1]
    t0=int(rows[a]['End_Timestamp']); t1=int(rows[b]['End_Timestamp'])
    busy=0; last=t0
    cat=defaultdict(float)
    for r in seg:
        s,e=int(r['Start_Timestamp']),int(r['End_Timestamp'])
        busy+=max(0,e-max(s,last)); last=max(last,e)
        n=r['Kernel_Name']
        k=('gemm' if ('Cijk' in n or 'fp8_gemm' in n) else 'attn' if 'attn' in n else 'adam' if 'adam' in n else 'other')
        cat[k]+=(e-s)/1e6
    print('step %.1f ms busy %.1f ms gaps %.1f ms'%((t1-t0)/1e6, busy/1e6, (t1-t0-busy)/1e6), {k:round(v,1) for k,v in cat.items()})
