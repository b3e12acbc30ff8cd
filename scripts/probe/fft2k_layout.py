# LDS bank model (as scripts/probe/stft_layout.py) for hz_fft2k.h's pass plan and the stationary
# engine's split / merge reads at bit-reversed positions, per candidate layout
from collections import Counter
N = 2048; T = 256
def br(x, lg=11): return int(bin(x)[2:].zfill(lg)[::-1], 2)
pats = []
pats += [('st', [t + 256 * i for t in range(T)]) for i in range(8)]
def dif(LD):
    return [[(((b >> LD) << (LD + 3)) + (b & ((1 << LD) - 1))) + (j << LD) for b in range(T)] for j in range(8)]
for LD in (6, 3, 0): pats += [('p%d' % LD, x) for x in dif(LD)]
split = []
for i in range(4):
    split.append(('sa%d' % i, [br(t + 256 * i) for t in range(T)]))
    split.append(('sb%d' % i, [br((2048 - (t + 256 * i)) & 2047) for t in range(T)]))
def cost(f, ps):
    tot = 0; worst = {}
    for name, addrs in ps:
        for h in range(0, T, 32):
            c = Counter(); seen = set()
            for e in addrs[h:h + 32]:
                if e in seen: continue
                seen.add(e); c[f(e) % 32] += 1
            m = max(c.values()); tot += m; worst[name] = max(worst.get(name, 0), m)
    return tot, worst
cands = {'none': lambda e: e, 'lx(e^((e>>3)&31))': lambda e: e ^ ((e >> 3) & 31)}
for s in range(2, 9):
    for t in range(0, 5):
        for m in (1, 3, 7, 15, 31):
            cands['xor s%d t%d m%d' % (s, t, m)] = (lambda s, t, m: (lambda e: e ^ (((e >> s) & m) << t)))(s, t, m)
for s in range(3, 8):
    for s2 in range(s + 1, 11):
        cands['xor2 %d %d' % (s, s2)] = (lambda a, b: (lambda e: e ^ ((e >> a) & 31) ^ ((e >> b) & 31)))(s, s2)
print('ideal passes', len(pats) * (T // 32), 'split', len(split) * (T // 32))
for k in ('none', 'lx(e^((e>>3)&31))'):
    print(k, cost(cands[k], pats), cost(cands[k], split)[0])
best = sorted((cost(f, pats)[0] * 4 + cost(f, split)[0], k) for k, f in cands.items())[:6]
for c, k in best: print(c, k, cost(cands[k], pats)[0], cost(cands[k], split)[0], cost(cands[k], split)[1])
