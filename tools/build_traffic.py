"""Per-kernel HBM bytes of one build (bench.py's live PMC passes: build_roofline.per_kernel) from a full
bench record: python tools/build_traffic.py gpurun_out/<tag>/bench_full.json"""
import json
import sys

d = json.load(open(sys.argv[1]))
for key in (None, "c2_bunny", "c5_merged_proxy_shadow"):
    rec = d if key is None else d.get(key)
    if not rec:
        continue
    n = (rec.get("config") or {}).get("tris") or rec.get("tris")
    br = rec["build_roofline"]
    print(f"{key or d['config']['config_id']}: {n} tris, build {rec['build_ms']:.4f} ms, traffic {br.get('traffic', 0) / 1e6:.2f} MB"
          f" = {br.get('traffic_over_bytes', 0):.2f}x the {br['bytes_per_tri']} B/tri model")
    for k, v in (br.get("per_kernel") or {}).items():
        r, w = v.get("read_x2", 0), v.get("write", 0)
        print(f"   {k:22s} read {r / 1e6:7.2f} MB ({r / n:6.1f} B/tri)  write {w / 1e6:7.2f} MB ({w / n:6.1f} B/tri)")
