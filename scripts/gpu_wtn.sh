# per-shape weight-gradient GEMMs: native TN vs hipBLASLt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4wtn}
mkdir -p $O
timeout -k 10 400 python scripts/bench_wgrad_tn.py > $O/w.log 2>&1 || { tail -20 $O/w.log; exit 1; }
grep -v amdgpu.ids $O/w.log
