"""One line per bench log: value, kernel time, options, K, index bytes, checks."""
import json
import sys

for f in sys.argv[1:]:
    for line in open(f, errors="replace"):
        if line.startswith("{"):
            d = json.loads(line)
            r = d["roofline"]
            c = d["config"]
            print(f"{f:40s} {d['value']:.3e} kern_us={r['avg_launch_ms'] * 1e3:7.1f} opts={c['load_options']:2d} "
                  f"K={c['deep_lut_k']} hbm={c['index_hbm_bytes'] / 1e9:5.1f}GB B={c['patterns_per_gpu']} "
                  f"m={c['pattern_len']} S={c.get('streams', 1)} G={c.get('batches_per_launch', 1)} NB={c.get('distinct_batches', '-')} {c.get('submit', 'py')} exact={d.get('parity', {}).get('bit_exact_vs_cpu')} self={d['self_location_check']}")
