O=gpurun_out
d() { tag=$1; shift; timeout -k 10 800 python tests/studies/kuhn_diag.py --hands 40000000 --every 10000000 "$@" > $O/kd_$tag.jsonl 2> $O/kd_$tag.err; echo "$tag rc=$?"; }
d lrbr01 --set lr_ar=0.005 --set lr_br=0.01 --set gamma=1.0 &
d lrbr002 --set lr_ar=0.005 --set lr_br=0.02 --set gamma=1.0 &
d lrbr01t50 --set lr_ar=0.005 --set lr_br=0.01 --set gamma=1.0 --set target_every=50 &
d lrbr01ar001 --set lr_ar=0.001 --set lr_br=0.01 --set gamma=1.0 &
d lrbr003ar02 --set lr_ar=0.02 --set lr_br=0.03 --set gamma=1.0 &
d eps02 --set lr_ar=0.005 --set lr_br=0.02 --set gamma=1.0 --set epsilon=0.2 &
wait
