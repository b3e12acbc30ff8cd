# LDS bank-conflict check of the 2048-point half-frame kernel's passes and gate walk (stft_half4096_kernel)
from collections import Counter
M=2048; T=256
pats=[]
def grp(ld):  # radix-8 pass on elements base + j*2^ld, base = ((b>>ld)<<(ld+3)) + (b & (2^ld-1))
    return [[(((b>>ld)<<(ld+3))+(b&((1<<ld)-1)))+(j<<ld) for b in range(T)] for j in range(8)]
for ld in (8,5,2): pats+=[('p%d'%ld,x) for x in grp(ld)]
pats+=[('c',[8*b+j for b in range(T)]) for j in range(8)]
def hib(x): return 1<<(x.bit_length()-1)
for i in range(4):
    qs=[];qp=[]
    for b in range(T):
        u=b+T*i
        if u>=M//2-1: u=M//2-2
        q=(u+1)+hib(u+1); qs.append(q); qp.append(q^(hib(q)-1))
    pats.append(('gq%d'%i,qs)); pats.append(('gp%d'%i,qp))
def cost(f):
    tot=0; worst={}
    for name,addrs in pats:
        for h in range(0,T,32):
            c=Counter(); seen=set()
            for e in addrs[h:h+32]:
                if e in seen: continue
                seen.add(e); c[f(e)%32]+=1
            m=max(c.values()); tot+=m; worst[name]=max(worst.get(name,0),m)
    return tot,worst
cands={'none':lambda e:e,'lx4096':lambda e:e^((e>>3)&31)}
for s in range(2,9):
  for t in range(0,5):
    for m in (1,3,7,15,31):
        cands['xor s%d t%d m%d'%(s,t,m)]=(lambda s,t,m:(lambda e:e^(((e>>s)&m)<<t)))(s,t,m)
print('ideal',len(pats)*(T//32))
print('lx4096',cost(cands['lx4096']))
for c,k in sorted((cost(f)[0],k) for k,f in cands.items())[:8]: print(c,k,cost(cands[k])[1])
