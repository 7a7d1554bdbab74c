exec(open(__import__('os').path.join(__import__('os').path.dirname(__file__), 'lds_bank_model.py')).read().split("print('dgrad A b128")[0])
def gemm_frag(KPAD):
    cs=[]
    for r0 in range(0,128,16):
        for kk in range(2):
            addrs=[((r0+(l&15))*KPAD+kk*32+8*(l>>4))*2 for l in range(64)]
            cs.append(cost(addrs,16,G128))
    return statistics.mean(cs)
def gemm_tr(RPAD):
    cs=[]
    for r0 in range(0,128,16):
        for kk in range(2):
            for half in range(2):
                addrs=[]
                for l in range(64):
                    q=(l&15)>>2; p=l&3; kb=kk*32+8*(l>>4)
                    addrs.append(((kb+4*half+q)*RPAD+r0+4*p)*2)
                cs.append(cost(addrs,8,G64))
    return statistics.mean(cs)
print('frag KPAD72', gemm_frag(72), 'KPAD64', gemm_frag(64), 'KPAD80', gemm_frag(80))
print('tr RPAD136', gemm_tr(136), 'RPAD128', gemm_tr(128), 'RPAD144', gemm_tr(144))
def gemm_frag_sw(sw):
    cs=[]
    for r0 in range(0,128,16):
        for kk in range(2):
            addrs=[]
            for l in range(64):
                r=r0+(l&15); ch=(kk*32+8*(l>>4))//8
                addrs.append((r*64+8*sw(r,ch))*2)
            cs.append(cost(addrs,16,G128))
    return statistics.mean(cs)
for name,sw in [('r&7',lambda r,c:c^(r&7)),('(r>>1)&7',lambda r,c:c^((r>>1)&7)),('r&3<<1', lambda r,c: c^((r&3)<<1)), ('mix', lambda r,c: c^((r&7)^((r>>3)&1)))]:
    print(name, gemm_frag_sw(sw))
# ds_write_b128 cost model: 8 groups of 8 contiguous lanes, bank (a/4)%32, data 16B per lane
G8=[list(range(i,i+8)) for i in range(0,64,8)]
def wcost(addrs):
    tot=0
    for g in G8:
        banks={}
        for l in g:
            a=addrs[l]
            for d in range(4):
                banks.setdefault((a//4+d)%32,set()).add(a//16)
        tot+=max(len(v) for v in banks.values())
    return tot
def stager_write(sw):
    cs=[]
    for i in range(4):
        addrs=[]
        for t in range(64):
            r=(t>>3)+32*i; ch=t&7
            addrs.append((r*64+8*sw(r,ch))*2)
        cs.append(wcost(addrs))
    return statistics.mean(cs)
print('write none', stager_write(lambda r,c:c), 'r&7', stager_write(lambda r,c:c^(r&7)))
def stager_write_pad(KPAD):
    cs=[]
    for i in range(4):
        addrs=[(((t>>3)+32*i)*KPAD+8*(t&7))*2 for t in range(64)]
        cs.append(wcost(addrs))
    return statistics.mean(cs)
print('write pad72', stager_write_pad(72))
