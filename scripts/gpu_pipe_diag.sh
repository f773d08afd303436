# GPU box (diagnostic): tables + optimizer state after each of 3 MF steps for the product split
# step and the pipelined step, compared bit for bit; then the pipelined-step tests.
set -o pipefail
mkdir -p gpurun_out
RG_PIPE=0 timeout -k 10 120 python scripts/pipe_dump.py gpurun_out/d_split.npz || exit $?
timeout -k 10 120 python scripts/pipe_dump.py gpurun_out/d_pipe.npz pipe || exit $?
python3 - <<'PY'
import numpy as np
a = np.load("gpurun_out/d_split.npz")
b = np.load("gpurun_out/d_pipe.npz")
n = 0
for k in a.files:
    x, y = a[k], b[k]
    if not np.array_equal(x, y):
        n += 1
        d = x != y
        rows = np.nonzero(d.reshape(d.shape[0], -1).any(1))[0] if d.ndim else []
        print("pipe", k, "differs:", len(rows), "rows, first", list(rows[:6]), "max", float(np.abs(x - y).max()))
print("pipe compared,", n, "arrays differ")
PY
