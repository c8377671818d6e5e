# the other configurations on the final tree: cfg1, cfg2-D64, cfg3, cfg5, drop-in
export TMPDIR=/tmp
bash tools/gpu_session.sh r06_s34 bench1 bench64 bench3 bench5 dropin || exit $?
O=gpurun_out/r06_s34
python - <<'PY'
import json
o = "gpurun_out/r06_s34"
for n in ("bench_cfg1", "bench_cfg2_d64", "bench_cfg3", "bench_cfg5", "bench_dropin"):
    d = json.loads([l for l in open(f"{o}/{n}.log") if l.startswith("{")][-1])
    r = d.get("roofline") or {}
    print(n, d["value"], d["ms_per_step"], d.get("step_ms_p10_p50_p90"), r.get("kernel"), r.get("frac"),
          (d.get("cpu_baseline") or {}).get("value"), d.get("gine_stack_ms_fwd_bwd"))
PY
