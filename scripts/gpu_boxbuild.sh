# GPU box, end of round: compile librg_hip.so ON the box (build(force=True) into the variant path
# _variants/librg_hip_boxbuild.so, the box's own hipcc), then run the GPU suite against it beside
# the shipped in-tree library.  Usage: bash scripts/gpu_boxbuild.sh TAG
set -o pipefail
TAG=${1:-final}
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
OUT=gpurun_out/boxbuild_$TAG.txt
hipcc --version 2>&1 | grep -i "HIP version" > $OUT
( while sleep 45; do echo "box build in progress"; done ) &
TICK=$!
timeout -k 10 900 python3 recommendation_gans_amd/build.py --force --variant boxbuild >> gpurun_out/boxbuild_log_$TAG.txt 2>&1
rc=$?
kill $TICK
[ $rc -eq 0 ] || { tail -20 gpurun_out/boxbuild_log_$TAG.txt; exit $rc; }
python3 - >> $OUT <<'PY'
import hashlib
for tag, p in (("box-built library", "recommendation_gans_amd/_variants/librg_hip_boxbuild.so"),
               ("shipped library  ", "recommendation_gans_amd/librg_hip.so")):
    print(tag, p, hashlib.sha256(open(p, "rb").read()).hexdigest()[:16])
PY
cat $OUT
RG_LIB=$R/recommendation_gans_amd/_variants/librg_hip_boxbuild.so timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_boxbuild_$TAG.log 2>&1
rc=$?; echo "boxbuild tests exit=$rc"; tail -3 gpurun_out/gpu_tests_boxbuild_$TAG.log
exit $rc
