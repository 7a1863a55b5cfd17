import sqlite3, statistics, sys
for path in sys.argv[1:]:
    db=sqlite3.connect(path)
    cur=db.cursor()
    ks=cur.execute("select d.start, d.end, s.kernel_name from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id=s.id order by d.start").fetchall()
    cs=cur.execute("select start, end, size from rocpd_memory_copy order by start").fetchall()
    ev=[(a,b,'K:'+n[:40]) for a,b,n in ks]+[(a,b,'C:%d'%sz) for a,b,sz in cs]
    ev.sort()
    multi=[e for e in ev if 'multi_vec' in e[2]]
    d=[(b-a)/1e3 for a,b,_ in multi]
    st=[a for a,b,_ in multi]
    per=[(st[i+1]-st[i])/1e3 for i in range(len(st)-1)]
    tc=[(b-a)/1e3 for a,b,n in ev if 'table_copy' in n]
    print(path, "multi_vec n=%d median dur %.2f us, start-to-start median %.2f us; table_copy_kernel n=%d median %.2f us" % (
        len(d), statistics.median(d), statistics.median(per), len(tc), statistics.median(tc) if tc else 0))
    i=[j for j,e in enumerate(ev) if 'multi_vec' in e[2]][60]
    t0=ev[i][0]
    for a,b,n in ev[i:i+7]:
        print("   %8.2f %8.2f %s"%((a-t0)/1e3,(b-t0)/1e3,n))
