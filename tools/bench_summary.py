"""One-line summary of a bench.py JSON line (tools/*.sh)."""
import json
import sys

j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
g = lambda k: (j.get(k) or {}).get("mrays_s")
print("C3", j["value"], "ms/step", j["ms_per_step"], "| C5", g("path_tracer_c5"), "| one-pass", g("one_pass_launches"),
      "| dopass", g("reference_dopass"), "| dopass-ahead", ((j.get("reference_dopass") or {}).get("render_ahead") or {}).get("mrays_s"), "| closest-shadow", g("closest_hit_shadows"), "| wpt", g("wavefront_tracer"),
      "| wpt-anyshadow", ((j.get("wavefront_tracer") or {}).get("shadow_any_hit") or {}).get("mrays_s"),
      "| camera", g("primary_rays"), "| c1", g("prim_tracer_c1"), "| binary", g("binary_bvh"),
      "| cpu", (j.get("cpu_baseline") or {}).get("value"),
      "| animate ms", (j.get("animation") or {}).get("ms_per_animate_median"))
