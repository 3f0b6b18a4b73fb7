#!/bin/bash
# Builds abvar/libog.so: oracle/ransac.c's five-point solver (up to oracle_five_point) as GPU device code.
set -e
cd "$(dirname "$0")/../.."
mkdir -p abvar /tmp/og_build
python3 - <<'PY'
s = open("oracle/ransac.c").read()
s = s[: s.index("/* ------------------------------------------------------------------ scoring (float32, explicit fma) */")]
s = s.replace("#include <math.h>\n#include <stdint.h>\n#include <stdlib.h>\n#include <string.h>\n", "")
s = s.replace("static int LL2Q[4][4], QL2C[10][4];\nstatic int tables_ready = 0;",
              "__device__ int LL2Q[4][4], QL2C[10][4];\n__device__ int tables_ready = 0;")
for t in ("LIN_E", "QUAD_E", "CUB_E"):
    s = s.replace("static const int " + t, "__device__ const int " + t)
# expose stage-1 intermediates: N (4 x 9) and the reduced rows 4..9, columns 10..19, as ransac.hip's stage buffer has them
s = s.replace("int oracle_five_point(const double* x1, const double* x2, double* Es) {",
              "int oracle_five_point(const double* x1, const double* x2, double* Es, double* dbgN, double* dbgR) {")
s = s.replace("    /* B(z): rows k = e - z f",
              "    if (dbgN) {\n        for (int k = 0; k < 4; ++k) for (int j = 0; j < 9; ++j) dbgN[9 * k + j] = N[k][j];\n"
              "        for (int r = 0; r < 6; ++r) for (int j = 0; j < 10; ++j) dbgR[10 * r + j] = A[4 + r][10 + j];\n    }\n"
              "    /* B(z): rows k = e - z f")
assert "dbgN[9 * k + j]" in s
open("/tmp/og_build/ransac_dev.c", "w").write(s)
PY
/opt/rocm/bin/hipcc -O3 -fPIC -shared --offload-arch=gfx950 -I/tmp/og_build tools/ubench/oracle_on_gpu.hip -o abvar/libog.so
echo built abvar/libog.so
