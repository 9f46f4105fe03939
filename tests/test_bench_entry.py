"""bench.py's own entry point at N = 2, exactly as a user or the driver types it
(`python bench.py --gpus 2 ...`, no launcher): bench.py must start the two ranks
itself and the printed line must describe a 2-rank job.  Runs on CPU with gloo
through the test-only --selftest hook (tiny oracle-quantised Llama, oracle
shard-local product); the greedy tokens must equal the unsharded model's."""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO


def _run(*extra, env_extra=None, timeout=300):
    env = dict(os.environ)
    env["PYTHONPATH"] = os.pathsep.join([REPO, os.path.join(REPO, "tests"), env.get("PYTHONPATH", "")])
    env.pop("WORLD_SIZE", None)
    env["OMP_NUM_THREADS"] = "1"
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--selftest", "bench_selftest_hook",
                           "--steps", "4", "--warmup", "1", "--prompt", "5", *extra],
                          capture_output=True, text=True, timeout=timeout, env=env, cwd=REPO)


def _line(p):
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, (p.stdout, p.stderr[-3000:])
    return json.loads(lines[0])


@pytest.mark.parametrize("extra,parallelism,gbatch", [((), "tp2-rowsplit-allgather", 1),
                                                      (("--weak",), "tp2-megatron-pair-allreduce", 2)])
def test_bench_gpus2_starts_two_ranks(extra, parallelism, gbatch):
    p = _run("--gpus", "2", *extra)
    assert p.returncode == 0, p.stderr[-4000:]
    line = _line(p)
    assert line["n_gpus"] == 2
    assert line["config"]["parallelism"] == parallelism
    assert line["config"]["global_batch"] == gbatch
    assert line["config"]["projection_groups"] == 4
    assert line["selftest"]["tokens_equal_unsharded"] is True


def test_bench_world_size_mismatch_exits_nonzero():
    """A launcher that started fewer ranks than --gpus asks for must not yield a line."""
    p = _run("--gpus", "2", env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert "WORLD_SIZE=1" in p.stderr


def test_greedy_token_is_torch_argmax():
    """The bench's two-stage greedy pick returns torch.argmax's index (the first maximal one),
    ties included, at the Llama-3 vocabulary and at a width it hands straight to argmax."""
    import torch
    sys.path.insert(0, REPO)
    from bench import greedy_token
    for seed in range(24):
        g = torch.Generator().manual_seed(seed)
        for V in (128256, 1000):
            x = torch.randn(2, 1, V, generator=g).half()
            if seed % 2:
                x = (x * 2).round().clamp(-3, 3)   # thousands of tied maxima
            assert torch.equal(greedy_token(x), x.argmax(-1))
