"""Test-only hook module for `bench.py --selftest bench_selftest_hook` (CPU, gloo):
the tiny oracle-quantised Linear4bit Llama (+ its unsharded dequantised reference)
and the shard-local product (oracle dequant + fp32 matmul).  Not part of the product."""
from test_distributed import _tiny_llama_4bit, _tp_hook


def tiny_model():
    return _tiny_llama_4bit()


local_matmul = _tp_hook
