# FIFO-refill simulation of apg_maze.hpp (CPU, numpy): PCG64 outputs consumed per DFS iteration of a
# 127 x 127 maze and the fraction of lane-iterations a refill rate / FIFO depth leaves short (uses maze_emu.py
# next to it).
import numpy as np
exec(open(__import__('os').path.join(__import__('os').path.dirname(__file__), 'maze_emu.py')).read().split("sys.path.insert")[0].replace("class R:","class R0:"))
# instrumented rng: count outputs consumed per DFS iteration
class R:
    def __init__(s,seed): s.g=np.random.default_rng(seed).bit_generator; s.has=0; s.u=0; s.used=0
    def n64(s): s.used+=1; return int(s.g.random_raw())
    def n32(s):
        if s.has: s.has=0; return s.u
        v=s.n64(); s.has=1; s.u=v>>32; return v&0xffffffff
    def dbl(s): return (s.n64()>>11)*(1.0/9007199254740992.0)
def trace(seed,h=127,w=127,bp=1.0):
    r=R(seed); ncx=(w-1)//2; ncy=(h-1)//2
    vis=np.zeros((ncy,ncx),bool); vis[0,0]=True
    stack=[]; cx=cy=0; k=0; first=True
    pidx=draw_perm(r); perm=perm_of(pidx); per=[]
    while True:
        u0=r.used
        E=0
        if cx+1<ncx and not vis[cy,cx+1]: E|=1
        if cx-1>=0 and not vis[cy,cx-1]: E|=2
        if cy+1<ncy and not vis[cy+1,cx]: E|=4
        if cy>0 and not vis[cy-1,cx]: E|=8
        pm=0
        for j in range(4): pm|=((E>>((perm>>(2*j))&3))&1)<<j
        pm&=(0xF<<k)&0xF
        if pm:
            j=(pm&-pm).bit_length()-1; d=(perm>>(2*j))&3; k=j+1
            take=first or r.dbl()<bp
            if take:
                nx=cx+(d==0)-(d==1); ny=cy+(d==2)-(d==3); vis[ny,nx]=True
                stack.append((cx,cy,perm,k)); cx,cy=nx,ny; first=True; k=0
                pidx=draw_perm(r); perm=perm_of(pidx)
        elif not stack: break
        else:
            cx,cy,perm,k=stack.pop(); first=False
        per.append(r.used-u0)
    return per
T=[trace(i*31+7) for i in range(6)]
print("outputs/iter", np.mean([np.mean(p) for p in T]), "max", max(max(p) for p in T))
for rate in (1,2):
  for D in (4,6,8,12):
    under=0; tot=0
    for p in T:
        c=0
        for need in p:
            for _ in range(rate):
                if c<D: c+=1
            if need>c: under+=1; c=0
            else: c-=need
            tot+=1
    print("rate",rate,"D",D,"underflow frac %.4f"%(under/tot))
