# Bench A/B of diagnostic libraries: for each name=path in LIBS ("default="
# = the shipped one) the bench with ARGS, ROUNDS times interleaved; prints
# the headline and kernel times of each run.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-libab}
mkdir -p "$OUT"
ARGS=${ARGS:-"--steps 20 --warmup 5 --cpu-baseline 0 --insitu 0 --ao 0 --frame 0 --ooc 0"}
for r in $(seq 1 ${ROUNDS:-2}); do
  for spec in ${LIBS:-default=}; do
    name=${spec%%=*}; path=${spec#*=}
    if [ -n "$path" ]; then export SPRAY_RT_LIB="$GRAFT_REPO_ROOT/$path"; else unset SPRAY_RT_LIB; fi
    timeout -k 10 300 python bench.py $ARGS > "$OUT/$name.$r.log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -5 "$OUT/$name.$r.log"; exit $rc; fi
    python3 - "$OUT/$name.$r.log" "$name" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
s = "%-10s step %.4f ms fused %.4f unfused %.4f + %.4f" % (sys.argv[2], d["ms_per_step"], d["kernels_ms"]["intersect_scene_shadow_pt"], d["kernels_ms"]["unfused"]["intersect_scene_spawn_pt"], d["kernels_ms"]["unfused"]["occluded_scene_masked"])
for k in ("ao", "ooc", "insitu", "frame"):
    if k in d:
        e = d[k]
        s += " | %s %.4f" % (k, e["ms_per_step"])
        if "roofline" in e: s += " (ah %.4f)" % e["roofline"]["avg_launch_ms"]
print(s)
PY
  done
done
