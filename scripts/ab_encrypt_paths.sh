# Encrypt kernel selection A/B (GPU box): quad vs lane over batch sizes, and
# the ragged / relay-stream layouts under the runtime's default choice.
# usage: bash scripts/ab_encrypt_paths.sh OUTDIR
O=${1:-gpurun_out/ab_enc}
mkdir -p "$O"
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread > "$O/pytest.log" 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_quad.py > "$O/ab_quad.txt" 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_ragged.py > "$O/ab_ragged.txt" 2>&1 || exit 1
echo done
