exec(open(__import__('os').path.join(__import__('os').path.dirname(__file__), 'lds_bank_model.py')).read().split("print('dgrad A b128")[0])
import collections
def c2f(XRS, tab=None, PW=13):
    cs=[]
    for mt in range(8):
        for ks in range(9):
            shift=(ks//3)*PW+ks%3
            addrs=[]
            for lane in range(64):
                r16=lane&15; q8=(lane>>4)*8
                if tab is None: mm=min(mt*16+r16,120)
                else:
                    mm=tab[mt*16+r16]; mm=0 if mm==255 else mm
                base=(mm//11)*PW+mm%11
                addrs.append(((base+shift)*XRS+q8)*2)
            cs.append(cost(addrs,16,G128))
    return statistics.mean(cs)
print('now', c2f(40))
for XRS in range(32,100,8): print(XRS, c2f(XRS))
def tiles(PW, S16, ntiles=8, npos=121, W=11):
    # residue class: slot parity structure for even S: residue mod 8 of base
    byres=collections.defaultdict(list)
    for m in range(npos):
        base=(m//W)*PW+m%W
        byres[(base*S16//2)%8 if S16%2==0 else base%16].append(m)
    A=[0,1,2,3,12,13,14,15]; B=list(range(4,12))
    T=[]
    for t in range(ntiles):
        tile=[None]*16
        for lanes in (A,B):
            for r in range(8):
                if byres[r]: tile[lanes[r]]=byres[r].pop(0)
        T.append(tile)
    left=[p for r in byres for p in byres[r]]
    for tile in T:
        for l in range(16):
            if tile[l] is None and left: tile[l]=left.pop(0)
    assert not left
    return [255 if p is None else p for t in T for p in t]
for XRS in (48,80,112):
    S16=XRS*2//16
    for PW in (13,14,15):
        T=tiles(PW,S16)
        print('balanced XRS',XRS,'PW',PW,c2f(XRS,T,PW))
