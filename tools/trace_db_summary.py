#!/usr/bin/env python3
"""Per-kernel totals, hardware-queue/stream mapping and busy-union of a
rocprofv3 --kernel-trace SQLite database (run_results.db): the check that
concurrent chains really overlap (union busy < summed kernel time)."""
import sqlite3, sys
from collections import defaultdict
for path in sys.argv[1:]:
    db=sqlite3.connect(path)
    cols=[r[1] for r in db.execute("pragma table_info(kernels)")]
    d=[dict(zip(cols,r)) for r in db.execute("select * from kernels")]
    d.sort(key=lambda x:x['start'])
    tot=defaultdict(lambda:[0,0.0]); qs=defaultdict(int)
    for x in d:
        t=tot[x['name'][:45]]; t[0]+=1; t[1]+=(x['end']-x['start'])/1e6
        qs[(x['queue_id'],x['stream_id'])]+=1
    print(path, "span ms", (d[-1]['end']-d[0]['start'])/1e6)
    for k,v in sorted(tot.items(), key=lambda kv:-kv[1][1])[:6]: print("  %-45s %6d %9.1f ms avg %.1f us"%(k,v[0],v[1],v[1]/v[0]*1e3))
    print("  queues/streams:", dict(qs))
    busy=0; cs=ce=None
    for x in d:
        if ce is None or x['start']>ce:
            if ce is not None: busy+=ce-cs
            cs,ce=x['start'],x['end']
        else: ce=max(ce,x['end'])
    busy+=ce-cs
    print("  union busy ms %.1f sum ms %.1f"%(busy/1e6, sum(x['end']-x['start'] for x in d)/1e6))
    # gaps: total idle between kernels
    print("  idle ms %.1f"%(((d[-1]['end']-d[0]['start'])-busy)/1e6))
