"""Audit the gemm4w dynamic tile queue in emitted ISA: for every returning global atomic, list each instruction that
touches its destination VGPR up to the LDS publish, and the vmcnt waits in between (profiles/r5_gemm_queue.md).

    hipcc -O3 -std=c++17 --offload-arch=gfx950 -S --offload-device-only csrc/kernels/gemm4w_00.hip -o /tmp/g00.s
    python3 tools/lab/queue_isa_audit.py /tmp/g00.s
"""
import re,sys
L=open(sys.argv[1]).read().split('\n')
def regs(tok):
    out=set()
    for m in re.finditer(r'\bv\[(\d+):(\d+)\]|\bv(\d+)\b',tok):
        if m.group(3): out.add(int(m.group(3)))
        else: out|=set(range(int(m.group(1)),int(m.group(2))+1))
    return out
for i,l in enumerate(L):
    if 'global_atomic_add' in l and ' sc0' in l:
        d=int(re.search(r'global_atomic_add v(\d+)',l).group(1))
        print('atomic at',i+1,'dst v%d'%d)
        for j in range(i+1,min(i+6000,len(L))):
            s=L[j].split(';')[0].strip()
            if not s or s.startswith('.') or s.endswith(':'): 
                if s.endswith(':'): print('   label',j+1,s)
                continue
            if 's_waitcnt' in s and 'vmcnt' in s: print('   wait',j+1,s)
            if d in regs(s):
                print('  USE',j+1,s); 
                if 'ds_write' in s: break
        print()
