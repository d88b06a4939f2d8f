O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_learner.py -x -q --timeout 200 --timeout-method thread -k "504 or 248" > $O/pytest_learner.log 2>&1 || { tail -30 $O/pytest_learner.log; exit 1; }
tail -1 $O/pytest_learner.log
d() { tag=$1; shift; timeout -k 10 800 python tests/studies/kuhn_diag.py --hands 40000000 --every 5000000 "$@" > $O/kd_$tag.jsonl 2> $O/kd_$tag.err; echo "$tag rc=$?"; }
d mse --quirks 504 &
d mse_lr --quirks 504 --set lr_ar=0.005 --set lr_br=0.02 --set gamma=1.0 &
d mse_def --quirks 504 --set lr_ar=0.1 --set lr_br=0.05 --set gamma=0.95 &
d mse1024 --quirks 504 --lanes 1024 &
wait
