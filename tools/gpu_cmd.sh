tools/gpu_steps.sh "parity:::500:::python -u -m pytest tests/test_gpu_parity.py -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread" "bench:::400:::python bench.py --steps 20"
