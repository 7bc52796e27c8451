mkdir -p gpurun_out/s28
timeout -k 10 400 python -u -m pytest tests/test_gpu.py tests/test_batcher.py -x -q --timeout 200 --timeout-method thread > gpurun_out/s28/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_ragged.py > gpurun_out/s28/ab_ragged.txt 2>&1 || exit 1
for g in 1 4 16 64; do echo "G=$g" >> gpurun_out/s28/ab_g.txt; CYAES_RAGGED_GROUP=$g timeout -k 10 300 python -u tools/ab_ragged.py >> gpurun_out/s28/ab_g.txt 2>&1 || exit 1; done
echo done
