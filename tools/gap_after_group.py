import sqlite3,sys
db=sqlite3.connect(sys.argv[1])
ks=db.execute("select name,start,end,queue_id from kernels order by start").fetchall()
for i,r in enumerate(ks):
    if 'gemm8_kernel<false, 1, 1>' in r[0]:
        nxt=[k for k in ks[i+1:] if k[3]==r[3]][:3]
        print(f"group {(r[2]-r[1])/1e3:7.1f} us; next on queue after", [(round((k[1]-r[2])/1e3,1), k[0][:30]) for k in nxt])
