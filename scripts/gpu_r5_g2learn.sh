cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5g2learn; mkdir -p $O
for v in native stock; do
  f=""; [ $v = stock ] && f="--stock"
  timeout -k 10 400 python scripts/gpt2_learning.py --rounds 200 --every 20 --lr 0.3 --mode sketch $f > $O/$v.log 2>&1 || { tail -20 $O/$v.log; exit 1; }
  echo $v; grep -o '"round": [0-9]*, "train_loss": [0-9.a-z]*, "val_nll": [0-9.]*' $O/$v.log
done
