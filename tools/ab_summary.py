import json,sys
for f in sys.argv[1:]:
    for l in open(f):
        if l.startswith("{"):
            d=json.loads(l); print(d["variant"],d["config"],d["frame"],d["trace_ms"],d["shade_ms"],d["tail_ms"],d["device_ms"],d["launches"],d["digest"][:8])
