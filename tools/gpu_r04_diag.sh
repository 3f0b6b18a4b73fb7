#!/bin/bash
# E-path exactness diagnostics: per-pair E / R differences and the first launch's five-point candidates vs the oracle.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 60 ./abvar/ns_steps > gpurun_out/r04_nssteps.log 2>&1; echo "ns_steps rc=$?"; tail -8 gpurun_out/r04_nssteps.log
timeout -k 10 60 ./abvar/ns_check > gpurun_out/r04_nscheck.log 2>&1; echo "ns_check rc=$?"; tail -6 gpurun_out/r04_nscheck.log
timeout -k 10 300 python -u tools/e_exact_diag.py > gpurun_out/r04_ediag.log 2>&1; rc=$?; echo "ediag rc=$rc"; tail -48 gpurun_out/r04_ediag.log
exit $rc
