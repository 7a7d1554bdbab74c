exec(open(__import__('os').path.join(__import__('os').path.dirname(__file__), 'lds_bank_model.py')).read().split("print('dgrad A b128")[0])
def win_pos(r,pw):
    w=r>>2;i=r&3
    return (2*(w>>2)+(i>>1))*pw+2*(w&3)+(i&1)
def c3_dgrad(PRS, tab=None, PW=12):
    cs=[]
    for mt in range(7):
        for ks in range(36):
            tapp=ks>>2; c0=(ks&3)*32; shift=(tapp//3)*PW+tapp%3
            addrs=[]
            for lane in range(64):
                r16=lane&15; q8=(lane>>4)*8
                if tab is None:
                    mm=min(mt*16+r16,99)
                else:
                    mm=tab[mt*16+r16]; mm=0 if mm==255 else mm
                base=(mm//10)*PW+mm%10
                addrs.append(((base+shift)*PRS+c0+q8)*2)
            cs.append(cost(addrs,16,G128))
    return statistics.mean(cs)
def c3_wgrad(drow, XRS):
    cD=[];cX=[]
    for wm in range(2):
     for ks in range(2):
      for i in range(4):
       for half in range(2):
        addrs=[]
        for lane in range(64):
            g16=lane&15; grp=lane>>4; q=g16>>2; p=g16&3
            kb=ks*32+grp*8; m0=(4*wm+i)*16
            addrs.append((drow(kb+4*half+q)+m0+4*p)*2)
        cD.append(cost(addrs,8,G64))
      for h in range(2):
       for wn in range(2):
        for j in range(9):
         for half in range(2):
          addrs=[]
          for lane in range(64):
            g16=lane&15; grp=lane>>4; q=g16>>2; p=g16&3
            kb=ks*32+grp*8
            x=win_pos(kb+4*half+q,10)
            n0=(18*h+9*wn+j)*16; tap=n0>>6; c0=n0&63; shift=(tap//3)*10+tap%3
            addrs.append(((x+shift)*XRS+c0+4*p)*2)
          cX.append(cost(addrs,8,G64))
    return statistics.mean(cD), statistics.mean(cX)
def c3_fwd(XRS):
    cs=[]
    for mt in range(4):
        for ks in range(18):
            tap=ks>>1; c0=(ks&1)*32; shift=(tap//3)*10+tap%3
            addrs=[]
            for lane in range(64):
                r16=lane&15; q8=(lane>>4)*8
                base=win_pos(4*(4*mt+(r16>>2))+(r16&3),10)
                addrs.append(((base+shift)*XRS+c0+q8)*2)
            cs.append(cost(addrs,16,G128))
    return statistics.mean(cs)
print('c3 dgrad now', c3_dgrad(136))
print('c3 wgrad now (D,X)', c3_wgrad(lambda r:r*136, 72))
print('c3 fwd now', c3_fwd(72))
for XRS in (64,72,80,88,96,112,144): print(' XRS',XRS,'wg X',c3_wgrad(lambda r:r*136, XRS)[1],'fwd',c3_fwd(XRS))
print('D blocked', c3_wgrad(lambda r:(r>>3)*1216+(r&7)*144, 80)[0])
# balanced tiles for c3 dgrad
def make_tiles3(PW=12, ntiles=7):
    byres={}
    for y in range(10):
        for x in range(10):
            byres.setdefault((y*PW+x)%8,[]).append(y*10+x)
    tiles=[[None]*16 for _ in range(ntiles)]
    A=[0,1,2,3,12,13,14,15]; B=list(range(4,12))
    left=[]
    for r in range(8):
        lst=byres[r]
        for t in range(ntiles):
            if lst: tiles[t][A[r]]=lst.pop(0)
            if lst: tiles[t][B[r]]=lst.pop(0)
        left+=lst
    for t in range(ntiles):
        for l in range(16):
            if tiles[t][l] is None and left: tiles[t][l]=left.pop(0)
    assert not left
    flat=[255 if p is None else p for t in tiles for p in t]
    assert sorted(x for x in flat if x!=255)==list(range(100))
    return flat
T3=make_tiles3()
for PRS in (136,144,176): print('c3 dgrad balanced PRS',PRS,c3_dgrad(PRS,T3))
print(','.join(map(str,T3)))
def c3_tilecost(PRS, tab, PW=12):
    out=[]
    for mt in range(7):
        cs=[]
        for ks in range(36):
            tapp=ks>>2; c0=(ks&3)*32; shift=(tapp//3)*PW+tapp%3
            addrs=[]
            for lane in range(64):
                r16=lane&15; q8=(lane>>4)*8
                mm=tab[mt*16+r16]; mm=0 if mm==255 else mm
                base=(mm//10)*PW+mm%10
                addrs.append(((base+shift)*PRS+c0+q8)*2)
            cs.append(cost(addrs,16,G128))
        out.append(statistics.mean(cs))
    return out
print(c3_tilecost(144,T3))
import collections
def make_tiles_best(PW, ntiles=7):
    byres=collections.defaultdict(list)
    for y in range(10):
        for x in range(10):
            byres[(y*PW+x)%8].append(y*10+x)
    tiles=[]
    A=[0,1,2,3,12,13,14,15]; B=list(range(4,12))
    for t in range(ntiles):
        tile=[None]*16
        for lanes in (A,B):
            for r in range(8):
                if byres[r]: tile[lanes[r]]=byres[r].pop(0)
        tiles.append(tile)
    left=[p for r in byres for p in byres[r]]
    for tile in tiles:
        for l in range(16):
            if tile[l] is None and left: tile[l]=left.pop(0)
    assert not left
    return [255 if p is None else p for t in tiles for p in t]
for PW in (12,13,14,15,16):
    cnt=collections.Counter((y*PW+x)%8 for y in range(10) for x in range(10))
    T=make_tiles_best(PW)
    print(PW, sorted(cnt.values()), c3_dgrad(144,T,PW), c3_tilecost(144,T,PW))
import random
def solve_tiles(PRS, PW, ntiles=7, iters=20000, seed=0):
    rnd=random.Random(seed)
    poss=list(range(100))
    rnd.shuffle(poss)
    slots=poss+[255]*(ntiles*16-100)
    def tcost(mt):
        return c3_tilecost_one(PRS, slots[mt*16:mt*16+16], PW)
    costs=[tcost(m) for m in range(ntiles)]
    for it in range(iters):
        i=rnd.randrange(len(slots)); j=rnd.randrange(len(slots))
        ti,tj=i//16,j//16
        if ti==tj or (slots[i]==255 and slots[j]==255): continue
        slots[i],slots[j]=slots[j],slots[i]
        ci,cj=tcost(ti),tcost(tj)
        if ci+cj<=costs[ti]+costs[tj]:
            costs[ti],costs[tj]=ci,cj
        else:
            slots[i],slots[j]=slots[j],slots[i]
    return statistics.mean(costs), slots
def c3_tilecost_one(PRS, tile, PW):
    cs=[]
    for ks in range(0,36,4):  # one c0 per tap is enough (c0 adds constant)
        tapp=ks>>2; shift=(tapp//3)*PW+tapp%3
        addrs=[]
        for lane in range(64):
            r16=lane&15; q8=(lane>>4)*8
            mm=tile[r16]; mm=0 if mm==255 else mm
            base=(mm//10)*PW+mm%10
            addrs.append(((base+shift)*PRS+q8)*2)
        cs.append(cost(addrs,16,G128))
    return statistics.mean(cs)
for PRS,PW in ((136,12),(136,13),(152,12),(144,12)):
    c,sl=solve_tiles(PRS,PW,iters=6000)
    print(PRS,PW,c)
T=make_tiles_best(12)
print('final', c3_dgrad(144,T,12), c3_tilecost(144,T,12))
print(','.join(map(str,T)))
