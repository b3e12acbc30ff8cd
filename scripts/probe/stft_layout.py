import itertools
N=4096; T=512
def bitrev(x,lg=12): return int(bin(x)[2:].zfill(lg)[::-1],2)
pats=[]
def dif(lh):
    ld=lh-2; out=[]
    for j in range(8):
        out.append([(((b>>ld)<<(lh+1))+(b&((1<<ld)-1)))+(j<<ld) for b in range(T)])
    return out
def dit(lh):
    out=[]
    for j in range(8):
        out.append([(((b>>lh)<<(lh+3))+(b&((1<<lh)-1)))+(j<<lh) for b in range(T)])
    return out
for lh in (11,8,5,2): pats+=[('dif%d'%lh,x) for x in dif(lh)]
for lh in (0,3,6,9): pats+=[('dit%d'%lh,x) for x in dit(lh)]
# gate: u = tid + 512 i, q = (u+1) + hibit(u+1), partner q' = q ^ (hibit(q)-1)
def hib(x): return 1<<(x.bit_length()-1)
for i in range(4):
    qs=[];qp=[]
    for b in range(T):
        u=b+512*i
        if u>=2047: u=2046
        q=(u+1)+hib(u+1); qs.append(q); qp.append(q^(hib(q)-1))
    pats.append(('gq%d'%i,qs)); pats.append(('gp%d'%i,qp))
def cost(f):
    tot=0; worst={}
    for name,addrs in pats:
        for h in range(0,T,32):
            banks=[f(e)%32 for e in addrs[h:h+32]]
            # distinct addresses per bank
            from collections import Counter
            c=Counter(); seen=set()
            for e,bk in zip(addrs[h:h+32],banks):
                if e in seen: continue
                seen.add(e); c[bk]+=1
            m=max(c.values()); tot+=m
            worst[name]=max(worst.get(name,0),m)
    return tot,worst
cands={}
cands['none']=lambda e:e
for s in range(2,8):
    for c in (1,2,4,8,16):
        cands['pad s%d c%d'%(s,c)]=(lambda s,c:(lambda e:e+(e>>s)*c))(s,c)
for s in range(3,10):
  for t in range(0,5):
    for m in (1,3,7,15,31):
        cands['xor s%d t%d m%d'%(s,t,m)]=(lambda s,t,m:(lambda e:e^(((e>>s)&m)<<t)))(s,t,m)
# two-term
for s1 in range(3,8):
  for s2 in range(s1+1,10):
    cands['pad2 %d %d'%(s1,s2)]=(lambda a,b:(lambda e:e+(e>>a)+(e>>b)))(s1,s2)
best=sorted((cost(f)[0],k) for k,f in cands.items())[:12]
ideal=len(pats)*(T//32)
print('ideal',ideal)
for c,k in best: print(c,k,cost(cands[k])[1])
