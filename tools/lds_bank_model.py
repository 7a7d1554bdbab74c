import statistics
G128=[list(range(0,4))+list(range(12,16))+list(range(20,28)), list(range(4,12))+list(range(16,20))+list(range(28,32))]
G128+=[[l+32 for l in g] for g in G128]
G64=[list(range(32)),list(range(32,64))]
def cost(addrs, width, groups):
    tot=0
    for g in groups:
        banks={}
        for l in g:
            a=addrs[l]
            for d in range(width//4):
                b=(a//4+d)%64
                banks.setdefault(b,set()).add(a//width)
        tot+=max(len(v) for v in banks.values())
    return tot
def tr_addr(row_of_lane, col0, RS):  # tr16: lane 4q+p in group g16 addresses row q, cols 4p
    pass
def conv2_dgrad(PRS, PW=15):
    cs=[]
    for mt in range(11):
        for ks in range(18):
            tapp=ks>>1; c0=(ks&1)*32; shift=(tapp//3)*PW+tapp%3
            addrs=[]
            for lane in range(64):
                r16=lane&15; q8=(lane>>4)*8
                mm=min(mt*16+r16,168); base=(mm//13)*PW+mm%13
                addrs.append(((base+shift)*PRS+c0+q8)*2)
            cs.append(cost(addrs,16,G128))
    return statistics.mean(cs)
def conv2_wgrad(DRS, XRS):
    cD=[];cX=[]
    for wm in range(4):
     for ks in range(4):
      for half in range(2):
        addrs=[]
        for lane in range(64):
            g16=lane&15; grp=lane>>4; q=g16>>2; p=g16&3
            kb=ks*32+grp*8
            addrs.append(((kb+4*half+q)*DRS+wm*16+4*p)*2)
        cD.append(cost(addrs,8,G64))
      for wn in range(2):
       for j in range(9):
        for half in range(2):
          addrs=[]
          for lane in range(64):
            g16=lane&15; grp=lane>>4; q=g16>>2; p=g16&3
            kb=ks*32+grp*8
            k=min(kb+4*half+q,120); x=(k//11)*13+k%11
            n0=(9*wn+j)*16; tap=n0>>5; c0=n0&31; shift=(tap//3)*13+tap%3
            addrs.append(((x+shift)*XRS+c0+4*p)*2)
          cX.append(cost(addrs,8,G64))
    return statistics.mean(cD), statistics.mean(cX)
print('dgrad A b128 (ideal 4):', conv2_dgrad(72))
print('wgrad D,X tr16 (ideal 2):', conv2_wgrad(72,40))
for PRS in range(64,137,8): print(' PRS',PRS,conv2_dgrad(PRS))
for DRS in range(64,137,8): print(' DRS',DRS,conv2_wgrad(DRS,40)[0])
for XRS in range(32,81,8): print(' XRS',XRS,conv2_wgrad(72,XRS)[1])
def conv2_dgrad_sw(PRS, sw, PW=15):
    cs=[]
    for mt in range(11):
        for ks in range(18):
            tapp=ks>>1; c0=(ks&1)*32; shift=(tapp//3)*PW+tapp%3
            addrs=[]
            for lane in range(64):
                r16=lane&15; q8=(lane>>4)*8
                mm=min(mt*16+r16,168); base=(mm//13)*PW+mm%13
                pos=base+shift; ch=(c0+q8)//8
                addrs.append((pos*PRS+ (sw(pos,ch))*8)*2)
            cs.append(cost(addrs,16,G128))
    return statistics.mean(cs)
for PRS in (64,72,80):
  for name,sw in [('none',lambda p,c:c),('x&7',lambda p,c:c^(p&7)),('x>>1&7',lambda p,c:c^((p>>1)&7)),('x&3',lambda p,c:c^(p&3)),('x>>1&3',lambda p,c:c^((p>>1)&3)), ('x*?',lambda p,c:c^((p*3)&7))]:
    if PRS!=64 and name!='none': 
        # only xor within 8 chunks when row has 8 chunks
        pass
    print(PRS,name,conv2_dgrad_sw(PRS,sw))
print('---')
print(sorted((conv2_wgrad(DRS,40)[0],DRS) for DRS in range(64,200,4))[:6])
print(sorted((conv2_wgrad(72,XRS)[1],XRS) for XRS in range(32,100,4))[:6])
print(sorted((conv2_dgrad(PRS),PRS) for PRS in range(64,200,8))[:6])
def dgrad_order(PRS, order, PW=15):
    cs=[]
    for mt in range(11):
        for ks in range(18):
            tapp=ks>>1; c0=(ks&1)*32; shift=(tapp//3)*PW+tapp%3
            addrs=[]
            for lane in range(64):
                r16=lane&15; q8=(lane>>4)*8
                idx=mt*16+r16
                oy,ox=order[min(idx,len(order)-1)]
                base=oy*PW+ox
                addrs.append(((base+shift)*PRS+c0+q8)*2)
            cs.append(cost(addrs,16,G128))
    return statistics.mean(cs)
raster=[(y,x) for y in range(13) for x in range(13)]
colmaj=[(y,x) for x in range(13) for y in range(13)]
blk=[]
for by in range(0,13,4):
  for bx in range(0,13,4):
    for y in range(by,min(by+4,13)):
      for x in range(bx,min(bx+4,13)): blk.append((y,x))
blk2=[]  # 2 rows x 8 cols blocks
for by in range(0,13,2):
  for bx in range(0,13,8):
    for y in range(by,min(by+2,13)):
      for x in range(bx,min(bx+8,13)): blk2.append((y,x))
for name,o in [('raster',raster),('colmaj',colmaj),('blk4x4',blk),('blk2x8',blk2)]:
    print(name, sorted((dgrad_order(PRS,o),PRS) for PRS in range(64,200,8))[:3])
import itertools
def assign(positions, PW=15):
    # positions: list of 16 (y,x) or None; return lane order (list of 16) s.t. lanes A={0-3,12-15} and B={4..11}
    # each cover distinct (pos mod 8)
    A=[0,1,2,3,12,13,14,15]; B=list(range(4,12))
    pos=[p for p in positions if p is not None]
    # bipartite-ish: try to split pos into two sets each with distinct residues mod 8
    res=lambda p: (p[0]*PW+p[1])%8
    bucket={}
    for p in pos: bucket.setdefault(res(p),[]).append(p)
    setA=[];setB=[]
    for r in range(8):
        lst=bucket.get(r,[])
        if len(lst)>=1: setA.append(lst[0])
        if len(lst)>=2: setB.append(lst[1])
        for extra in lst[2:]: setB.append(extra)  # conflict, unavoidable
    rest=[p for p in pos if p not in setA and p not in setB]
    order=[None]*16
    # fill dummies with residues missing
    for i,l in enumerate(A):
        order[l]=setA[i] if i<len(setA) else None
    for i,l in enumerate(B):
        order[l]=setB[i] if i<len(setB) else None
    return order
def dgrad_perm(PRS, PW=15):
    cs=[]
    tiles=[]
    for mt in range(11):
        ps=[raster[i] if i<169 else None for i in range(mt*16,mt*16+16)]
        tiles.append(assign(ps,PW))
    for mt in range(11):
        for ks in range(18):
            tapp=ks>>1; c0=(ks&1)*32; shift=(tapp//3)*PW+tapp%3
            addrs=[]
            for lane in range(64):
                r16=lane&15; q8=(lane>>4)*8
                p=tiles[mt][r16]
                if p is None: p=(0,0)
                base=p[0]*PW+p[1]
                addrs.append(((base+shift)*PRS+c0+q8)*2)
            cs.append(cost(addrs,16,G128))
    return statistics.mean(cs), tiles
for PRS in (80,112,144,176):
    print(PRS, dgrad_perm(PRS)[0])
c,t=dgrad_perm(80)
mt=2
for grp in G128[:2]:
    sl=[]
    for l in grp:
        r16=l&15; q8=(l>>4)*8; p=t[mt][r16]; base=p[0]*15+p[1]
        a=((base)*80+q8)*2
        sl.append(((a//16)%16, r16, base%8, q8))
    print(sorted(sl))
def make_tiles(PW=15, ntiles=11):
    byres={}
    for y in range(13):
        for x in range(13):
            byres.setdefault((y*PW+x)%8,[]).append((y,x))
    tiles=[[None]*16 for _ in range(ntiles)]
    A=[0,1,2,3,12,13,14,15]; B=list(range(4,12))
    leftovers=[]
    for r in range(8):
        lst=byres[r]
        for t in range(ntiles):
            if lst: tiles[t][A[r]]=lst.pop(0)
            if lst: tiles[t][B[r]]=lst.pop(0)
        leftovers+=lst
    # fill remaining None slots with leftovers
    for t in range(ntiles):
        for l in range(16):
            if tiles[t][l] is None and leftovers: tiles[t][l]=leftovers.pop(0)
    assert not leftovers
    return tiles
def eval_tiles(tiles, PRS, PW=15):
    cs=[]
    for mt in range(len(tiles)):
        for ks in range(18):
            tapp=ks>>1; c0=(ks&1)*32; shift=(tapp//3)*PW+tapp%3
            addrs=[]
            for lane in range(64):
                r16=lane&15; q8=(lane>>4)*8
                p=tiles[mt][r16] or (0,0)
                addrs.append(((p[0]*PW+p[1]+shift)*PRS+c0+q8)*2)
            cs.append(cost(addrs,16,G128))
    return statistics.mean(cs)
T=make_tiles()
print('balanced tiles PRS80', eval_tiles(T,80), [sum(1 for p in t if p) for t in T])
flat=[]
for t in T:
    for p in t: flat.append(255 if p is None else p[0]*13+p[1])
print(len(flat), sorted(x for x in flat if x!=255)==list(range(169)))
print(','.join(map(str,flat)))
