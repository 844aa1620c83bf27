import sqlite3,glob,sys
f=sorted(glob.glob(sys.argv[1]+'/**/*.db',recursive=True))[-1]
c=sqlite3.connect(f)
for r in c.execute("select name, count(*), avg(end-start)/1000.0 from kernels group by name order by sum(end-start) desc").fetchall()[:24]:
    print(r[0][:60], r[1], round(r[2],2))
