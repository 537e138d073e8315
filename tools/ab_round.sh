# Same-box A/B of a whole round: the previous round's tree and HEAD, alternating bench runs (GPU).
#   git worktree add -f _r4end <previous round's last commit>; make -C _r4end/show-attend-and-tell_amd/csrc
#   gpurun -- 'bash tools/ab_round.sh'            (logs under gpurun_out/r5_s30/)
set -u
O=gpurun_out/r5_s30; mkdir -p $O
A="--steps 150 --no-cpu-baseline --fp32-steps 0 --no-diagnostics"
run() { echo "[$(date +%T)] $1"; }
run old1; (cd _r4end && timeout -k 10 300 python bench.py $A) > $O/old1.log 2>&1 || exit $?
run new1; timeout -k 10 300 python bench.py $A > $O/new1.log 2>&1 || exit $?
run old2; (cd _r4end && timeout -k 10 300 python bench.py $A) > $O/old2.log 2>&1 || exit $?
run new2; timeout -k 10 300 python bench.py $A > $O/new2.log 2>&1 || exit $?
run old_cfg5; (cd _r4end && timeout -k 10 300 python bench.py $A --bert --network vgg19) > $O/old_cfg5.log 2>&1 || exit $?
run new_cfg5; timeout -k 10 300 python bench.py $A --bert --network vgg19 > $O/new_cfg5.log 2>&1 || exit $?
for f in old1 new1 old2 new2 old_cfg5 new_cfg5; do python - $O/$f.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1]); print(sys.argv[1], d["value"], d["ms_per_step"])
PY
done
