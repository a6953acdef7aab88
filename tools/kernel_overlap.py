import csv, collections, sys
rows=list(csv.DictReader(open(sys.argv[1])))
rows=[r for r in rows if 'span_decode' in r['Kernel_Name'] or 'fixed_group' in r['Kernel_Name']]
print(collections.Counter(r['Queue_Id'] for r in rows))
ks=sorted((int(r['Start_Timestamp']),int(r['End_Timestamp'])) for r in rows)
ov=sum(1 for i in range(1,len(ks)) if ks[i][0] < ks[i-1][1])
tot=ks[-1][1]-ks[0][0]; busy=sum(b-a for a,b in ks)
print("overlapping", ov, "of", len(ks), "span", tot/1e3, "us; sum kernel", busy/1e3, "mean", busy/len(ks)/1e3)
