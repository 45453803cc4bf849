import os, sys, numpy as np
R=os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0,R+'/oracle'); sys.path.insert(0,R+'/tests'); sys.path.insert(0,R+'/bwa-mem2-arm_amd/py')
import oracle, bsw
from test_fmi import sample_reads
ref=np.random.default_rng(9).integers(0,4,200_000,dtype=np.uint8)
reads,off,lens=sample_reads(ref,300,151,21)
o=oracle.FmiRef(ref); f=bsw.Fmi(ref)
oo,oc=o.collect_intv(reads,off,lens,cap=320)
go,gc=f.collect_intv(reads,off,lens,cap=320)
bad=0
for i in range(len(lens)):
    a=[(int(v['k']),int(v['l']),int(v['s']),int(v['info']>>32),int(v['info']&0xffffffff)) for v in oo[i,:oc[i]]]
    b=[(int(v['k']),int(v['l']),int(v['s']),int(v['info']>>32),int(v['info']&0xffffffff)) for v in go[i,:gc[i]]]
    if a!=b:
        bad+=1
        if bad<4: print(i,'\nwant',a,'\ngot ',b, '\nN at', list(np.nonzero(reads[off[i]:off[i]+lens[i]]==4)[0]))
print('bad',bad)
