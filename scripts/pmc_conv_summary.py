import csv,collections,re,sys
for d in sys.argv[1:]:
    agg=collections.defaultdict(lambda: collections.defaultdict(float)); disp=collections.defaultdict(set); dur={}
    for r in csv.DictReader(open(d+'/run_counter_collection.csv')):
        k=r['Kernel_Name'].replace('void ','').replace('(anonymous namespace)::','').replace('commeff::','').split('(')[0]
        if 'conv' not in k: continue
        agg[k][r['Counter_Name']]+=float(r['Counter_Value']); disp[k].add(r['Dispatch_Id'])
        dur[(k,r['Dispatch_Id'])]=int(r['End_Timestamp'])-int(r['Start_Timestamp'])
    print('==',d)
    for k,v in sorted(agg.items()):
        n=len(disp[k]); us=sum(t for (kk,_),t in dur.items() if kk==k)/n/1e3
        cf=v['SQ_LDS_BANK_CONFLICT']/max(1,v['SQ_LDS_IDX_ACTIVE'])*100
        print(f"{k[:60]:60s} n={n:3d} us={us:7.1f} ldscf={cf:5.1f}% wait={v['SQ_WAIT_ANY']/max(1,v['SQ_WAVE_CYCLES'])*100:5.1f}%")
