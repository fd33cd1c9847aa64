import sys,json
from collections import defaultdict
d=defaultdict(list)
for l in open(sys.argv[1]):
    if not l.startswith("{"): continue
    j=json.loads(l); d[j["variant"]].append((j["shade_ms"],j["trace_ms"],j["device_ms"],j["slots"],j["digest"]))
for k,v in d.items():
    sh=sorted(x[0] for x in v); print(k, "shade", sh, "trace mean %.2f" % (sum(x[1] for x in v)/len(v)), "dev mean %.2f" % (sum(x[2] for x in v)/len(v)), set(x[3] for x in v), set(x[4] for x in v))
