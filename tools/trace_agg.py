import csv,re,sys,collections
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
# steps: count of sgd kernels
idx=[i for i,r in enumerate(rows) if 'sgd_flat' in r['Kernel_Name']]
# take last N steps between sgd kernels
n=int(sys.argv[2]) if len(sys.argv)>2 else 3
seg=rows[idx[-n-1]+1:idx[-1]+1]
agg=collections.defaultdict(lambda:[0,0.0])
tot=0
for r in seg:
    k=r['Kernel_Name']
    k=re.sub(r'\(anonymous namespace\)::','',k)
    m=re.search(r'(\w+_kernel(<[^()]*>)?|Cijk\w{0,40}|oneRankReduce|copyBuffer|fillBuffer\w*|FillFunctor|elementwise_kernel<[^>]*>|\w+Functor\w*)',k)
    name=m.group(1) if m else k[:60]
    d=(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1000
    agg[name][0]+=1; agg[name][1]+=d; tot+=d
win=(int(seg[-1]['End_Timestamp'])-int(seg[0]['Start_Timestamp']))/1000/n
print(f"per step: window {win:.1f} us, busy {tot/n:.1f} us, kernels {len(seg)/n:.0f}")
for k,(c,d) in sorted(agg.items(),key=lambda x:-x[1][1])[:int(sys.argv[3]) if len(sys.argv)>3 else 30]:
    print(f"{d/n:9.1f} us {c/n:6.1f}x {d/c:8.1f} avg  {k[:90]}")
