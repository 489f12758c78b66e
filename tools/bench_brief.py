"""One-screen summary of a bench.py JSON line: python tools/bench_brief.py FILE"""
import json
import sys

d = json.loads([ln for ln in open(sys.argv[1]) if ln.startswith("{")][-1])
r = d["roofline"]
print(f"headline {d['value'] / 1e9:.2f} Gbit/s  {d['ms_per_step']:.3f} ms/step  kernel {r['kernel_ms']:.3f} ms "
      f"call {r.get('call_ms', 0):.3f} ms  {r['bound']} frac {r['frac']:.3f}  nominal {r.get('nominal_frac', 0):.3f}  "
      f"hbm {r.get('hbm_frac_measured', 0):.3f}  fer {d['fer']}  sum_it {d['sum_iterations']}")
if "end_to_end" in d:
    print(f"end_to_end {d['end_to_end']['value'] / 1e9:.2f} Gbit/s {d['end_to_end']['ms_per_step']:.3f} ms")
for k, v in d.get("variants", {}).items():
    print(f"variant {k}: kernel {v['kernel_ms']:.3f} ms  call {v.get('call_ms', 0):.3f}  fer {v['fer']}  "
          f"bound {v['roofline']['bound']}")
for p in d.get("config3_sweep", {}).get("points", []):
    print(f"c3 q={p['qber_nominal']:.2f} {p['ms']:.2f} ms fer {p['fer']:.4f} it {p['mean_iterations']:.3f} "
          f"ref {p['reference']['mean_it']}/{p['reference']['fer']} ok={p['matches_reference']}")
if "config4" in d:
    c = d["config4"]
    print(f"c4 {c['frames']} frames on {c['n_gpus']} GPU(s): {c['value'] / 1e9:.2f} Gbit/s {c['ms']:.2f} ms "
          f"fer {c['fer']} sum_it {c['sum_iterations']} matches_fixture {c['matches_fixture']}")
if "cpu_baseline" in d:
    c = d["cpu_baseline"]
    print(f"cpu {c['value'] / 1e6:.1f} Mbit/s on {c['cores']} threads; all-core est "
          f"{c['all_cores_estimate']['value'] / 1e6:.1f} on {c['all_cores_estimate']['cores']}")
