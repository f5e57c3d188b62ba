#!/usr/bin/env python3
"""Per-round device latency of the device-elimination headline from rocprofv3
kernel + memory-copy traces: trace_rounds.py DIR... (each DIR holds run_kernel_trace.csv
and run_memory_copy_trace.csv, e.g. from tools/r6_trace_libs.sh)."""
import csv, sys, statistics
def rounds(d):
    ks=list(csv.DictReader(open(d+'/run_kernel_trace.csv')))
    cs=list(csv.DictReader(open(d+'/run_memory_copy_trace.csv')))
    ev=[(int(r['Start_Timestamp']),int(r['End_Timestamp']),r['Kernel_Name'].split('(')[0].replace('sgpu::',''),int(r['Grid_Size_X'])) for r in ks]
    ev+=[(int(r['Start_Timestamp']),int(r['End_Timestamp']),'CPY',0) for r in cs if 'HOST_TO_DEVICE' in r['Direction']]
    ev.sort()
    # a round: from a k_ge (big) start - find the preceding copy start; to the k_hostcopy after the solve_main
    lat=[]; gexec=[]
    for i,(s,e,n,g) in enumerate(ev):
        if n=='k_ge' and g>512:
            # first copy start within 200us before
            c0=min([x[0] for x in ev[max(0,i-4):i+3] if x[2]=='CPY' and abs(x[0]-s)<300000] or [s])
            # first exec after
            ex=next((x for x in ev[i+1:i+12] if x[2]=='k_exec'),None)
            sm=next((x for x in ev[i+1:i+20] if x[2]=='k_solve_main'),None)
            if ex and sm:
                lat.append((sm[1]-c0)/1e3); gexec.append((ex[0]-c0)/1e3)
    return lat, gexec
for d in sys.argv[1:]:
    lat,gx=rounds(d)
    print(d, 'rounds', len(lat), 'median copy->solve_main end %.1f us'%statistics.median(lat), 'median copy->first exec %.1f us'%statistics.median(gx))
