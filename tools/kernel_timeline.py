import csv,glob,sys
f=glob.glob(sys.argv[1]+'/**/*kernel_trace.csv',recursive=True)[0]
rows=list(csv.DictReader(open(f)))
ks=sorted((int(r["Start_Timestamp"]),int(r["End_Timestamp"]),r["Kernel_Name"]) for r in rows)
idx=[i for i,k in enumerate(ks) if "rollout_chunk_kernel" in k[2]]
for j in idx[-3:]:
    t0=ks[j][0]; i=j
    print("---")
    while i < len(ks) and (i==j or "rollout_chunk" not in ks[i][2]):
        s,e,n=ks[i]; print(f"{(s-t0)/1e3:9.1f} +{(e-s)/1e3:7.1f} gap {(s-ks[i-1][1])/1e3:7.1f} {n[:80]}"); i+=1
