import sys; sys.path.insert(0,'/root/repo/tests')
import scenario_lib as S
cases = [("C1",S.CONFIGS["C1"]),("C1var",S.CONFIGS["C1var"]),("C2x16",S.replace(S.CONFIGS["C2"],streams=16)),
         ("C4x16",S.replace(S.CONFIGS["C4"],streams=16)),("C3x1500",S.replace(S.CONFIGS["C3"],originals=1500))]
lib = S.AMD_LIB if len(sys.argv)>1 and sys.argv[1]=="amd" else S.SIM_LIB
tot=0
for name,cfg in cases:
  for hd in (1,0):
    c=S.replace(cfg, hash_data=hd)
    ref,_,_=S.run_capi(S.REF_LIB,c)
    b,rep=S.run_batch(lib,c,verify=True)
    bad=[i for i in range(c.streams) if ref[i].digest!=b[i].digest or ref[i].status!=b[i].status]
    tot+=len(bad)
    print(name,"hash",hd,"mismatch",len(bad),"rounds",rep.rounds,"checked",rep.checked,"mm",rep.mismatches,"status",S.summary(b)["status"],flush=True)
print("TOTAL",tot)
import sys as _s
_s.exit(1 if tot else 0)
