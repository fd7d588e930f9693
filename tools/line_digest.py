"""One-line digest of a bench.py JSON line (tools/gpu.sh): headline, config 4 (with its per-step
record), config 5, WAL, end-to-end, footprint."""
import json
import sys

d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
out = []
m = lambda v: round(v / 1e6, 2)
if "config4" in d or d.get("unit") == "sigs/s":
    out.append(f"c2 {m(d['value'])} M/s ok={d['correct']} frac={d.get('roofline', {}).get('frac')} "
               f"prep_ms={d.get('roofline', {}).get('kernel_ms')}")
    if d.get("sustained"):
        out.append(f"sust {m(d['sustained']['median'])}")
    if d.get("end_to_end"):
        out.append(f"e2e {m(d['end_to_end']['value'])} ({round(d['end_to_end']['value'] / d['value'], 3)})")
c4 = d.get("config4") or (d if "blocks/s" in str(d.get("unit")) else None)
if c4:
    s = c4.get("step_ms", {})
    out.append(f"c4 {m(c4['value'])} M blk/s ms/step={c4['ms_per_step']} steps={c4.get('steps')} "
               f"dev={s.get('device')} host={s.get('host_enqueue')} stages={c4.get('pipeline', {}).get('stage_ms')}")
    if c4.get("host_fed"):
        h = c4["host_fed"]
        out.append(f"hostfed {m(h['value'])} ({h['frac_of_pcie_bound']} of PCIe) pageable {m(h['pageable'])}")
c5 = d.get("config5") or (d if "shapes" in d else None)
if c5:
    for k, v in c5["shapes"].items():
        c = v["concurrent_1_block_callers"]
        out.append(f"c5 {k} p50={v['gpu']['p50_us']} p99={v['gpu']['p99_us']} conc={c['gpu']['blocks_per_s']} "
                   f"p50c={c['gpu']['p50_us']} cpp={c['gpu'].get('calls_per_device_pass')} onl={c['gpu'].get('online_requests')}/{c['gpu'].get('online_launches')} cpu={c.get('cpu_own_core', {}).get('blocks_per_s')}")
        f = v.get("fan_in_callers")
        if f:
            out.append(f"fanin{f['callers']} {k} gpu={f['gpu']['blocks_per_s']} p50={f['gpu']['p50_us']} "
                       f"p99={f['gpu']['p99_us']} cpu={f.get('cpu_own_core', {}).get('blocks_per_s')}")
w = d.get("wal") or (d if "WAL" in d.get("metric", "") else None)
if w:
    out.append(f"wal {w['value']} GB/s stages={w.get('stage_ms')}")
if d.get("footprint"):
    out.append("fp " + " ".join(f"r{x['rank']}:rss={x['host_rss_peak_GB']}G,hbm={x['hbm_peak_GB']}G" for x in d["footprint"]["per_rank"]))
print(" | ".join(out))
