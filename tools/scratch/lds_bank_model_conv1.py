XC_W=32; XC_SZ=30*32
groups=[list(range(0,4))+list(range(12,16))+list(range(20,28)), list(range(4,12))+list(range(16,20))+list(range(28,32))]
groups+= [[l+32 for l in g] for g in groups]
def cost(addrs):  # addrs: byte addr per lane (64), b128
    tot=0
    for g in groups:
        banks={}
        for l in g:
            a=addrs[l]
            for d in range(4):
                b=(a//4+d)%64
                banks.setdefault(b,set()).add(a//16)
        tot+=max(len(v) for v in banks.values())
    return tot
import statistics
cs=[]
for mt in range(43):
    addrs=[]
    for lane in range(64):
        r16=lane&15; gq=lane>>4
        w=min(4*mt+(r16>>2),168); i=r16&3
        oh=2*(w//13)+(i>>1); ow=2*(w%13)+(i&1)
        e=(ow&7)*XC_SZ+oh*XC_W+(ow&~7)+gq*XC_W
        addrs.append(e*2)
    cs.append(cost(addrs))
print('fwd A read cycles per instr: mean',statistics.mean(cs),'min',min(cs),'max',max(cs),' (ideal 4)')
def fwd_cost(RS, CS, perm=None):
    cs=[]
    for mt in range(43):
        addrs=[]
        for lane in range(64):
            r16=lane&15; gq=lane>>4
            wi=4*mt+(r16>>2)
            w=min(wi,168) if perm is None else perm(wi)
            i=r16&3
            oh=2*(w//13)+(i>>1); ow=2*(w%13)+(i&1)
            e=(ow&7)*CS+oh*RS+(ow&~7)+gq*RS
            addrs.append(e*2)
        cs.append(cost(addrs))
    return statistics.mean(cs)
best=[]
for RS in range(32,49,8):
    for CS in range(30*RS, 30*RS+8*40, 8):
        best.append((fwd_cost(RS,CS),RS,CS))
best.sort(); print(best[:10])
def wg_cost(RS, CS):
    tot=[]
    for ks in range(26):
        for nt in range(2):
            addrs=[]
            for lane in range(64):
                i16=lane&15; g=lane>>4; t=nt*16+i16
                if t>=25: t=0
                e=(t%5)*CS+(t//5+ks)*RS+8*g
                addrs.append(e*2)
            tot.append(cost(addrs))
    return statistics.mean(tot)
print('wgrad B', wg_cost(32,960), wg_cost(32,1048), wg_cost(32,1176))
for CS in (960,1048,1176): print(CS, fwd_cost(32,CS))
r=[]
for RS in (32,40,48):
  for CS in range(30*RS, 30*RS+8*64, 8):
    r.append((wg_cost(RS,CS)+fwd_cost(RS,CS)*86/52/2, wg_cost(RS,CS), fwd_cost(RS,CS), RS, CS))
r.sort(); print(r[:8])
for RS in (32,40,48):
  r=sorted((wg_cost(RS,CS),CS) for CS in range(30*RS, 30*RS+8*64, 8))
  print('wg',RS,r[:3])
