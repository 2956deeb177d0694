cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5ab4; mkdir -p $O
cat > /tmp/rs.py <<'PY'
import sys, torch
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import test_fedavg_native as t
from commefficient_amd.models.fixup import ResNet18
for extra in (["--fedavg_batch_size", "-1", "--num_fedavg_epochs", "2"], ["--fedavg_batch_size", "2", "--num_fedavg_epochs", "1"]):
    torch.manual_seed(0)
    base = ResNet18(num_classes=100)
    G, n = 6, 5
    _, _, b_n, _ = t._round(base, "native", "bf16", G, n, extra)
    _, _, b_v, _ = t._round(base, "vmap", "bf16", G, n, extra)
    _, _, b_vf, _ = t._round(base, "vmap", "fp32", G, n, extra)
    worst = []
    for k in b_v:
        if "running" in k:
            ref = b_vf[k].norm().item()
            worst.append(((b_n[k] - b_vf[k]).norm().item() / ref, (b_v[k] - b_vf[k]).norm().item() / ref,
                          (b_n[k] - b_vf[k]).abs().max().item(), (b_v[k] - b_vf[k]).abs().max().item(), k))
    worst.sort(reverse=True)
    for w in worst[:4]: print(extra[1], "rel_n %.4f rel_v %.4f max_n %.3f max_v %.3f %s" % w)
PY
for v in new old; do
if [ $v = old ]; then export COMMEFF_BN_OLDCB=1; fi
echo "== $v"; timeout -k 10 300 python -u /tmp/rs.py > $O/$v.log 2>&1; echo "rc=$?"; tail -8 $O/$v.log
done
