# GPU box, end of round 3: a fresh hipcc build of the library ON the box (variant
# _variants/librg_hip_boxbuild.so) and the whole GPU suite against it, then the shipped
# library: every gpu test, smoke, driver-shaped benches, kernel-trace profiles, the PMC
# traffic of the dense pass and every bench mode (scripts/gpu_final.sh).
# Usage: bash scripts/gpu_final_r3.sh TAG
set -o pipefail
TAG=${1:-r3}
mkdir -p gpurun_out
export TMPDIR=/tmp
(while sleep 20; do date >> gpurun_out/heartbeat_$TAG.txt; done) & HB=$!
timeout -k 10 900 python -c "
import hashlib, os, subprocess
from recommendation_gans_amd import build
p = build.build(variant='boxbuild')
h = lambda f: hashlib.sha256(open(f, 'rb').read()).hexdigest()[:16]
print('hipcc:', subprocess.run([build._hipcc(), '--version'], capture_output=True, text=True).stdout.splitlines()[0])
print('box-built library', os.path.relpath(p), h(p))
print('shipped library  ', os.path.relpath(build.LIB), h(build.LIB))
" > gpurun_out/boxbuild_$TAG.txt 2>&1; rc=$?
kill $HB
cat gpurun_out/boxbuild_$TAG.txt; [ $rc -eq 0 ] || exit $rc
RG_LIB=$PWD/recommendation_gans_amd/_variants/librg_hip_boxbuild.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_boxbuild_$TAG.log 2>&1
rc=$?; echo "box-build tests exit=$rc"; tail -3 gpurun_out/gpu_tests_boxbuild_$TAG.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_final.sh $TAG
