set -u
O=gpurun_out/r06_probe; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_xgmi_gpu.py tests/test_elastic_gpu.py > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 2 --oversubscribe --dist-backend gloo --steps 20 --warmup 5 --ingest local > $O/bench2_mlp.json 2> $O/bench2_mlp.err || exit 4
tail -1 $O/bench2_mlp.json | cut -c1-300
grep -i "probe\|xgmi" $O/bench2_mlp.err | head -5
