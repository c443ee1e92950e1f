"""bench.py's N > 1 branch on the one-GPU test box: `bench.py --gpus 2` starts torch.distributed.run itself (no external
launcher), the two ranks build the DDP step (bucketed gradient all-reduce on the side stream, SyncBN), time the same
number of steps between barriers and report the MAX-over-ranks elapsed time from rank 0 as ONE JSON line.  RCCL needs a
GPU per rank, so the test runs the ranks over gloo on the same GPU (SSSEG_BENCH_BACKEND=gloo); the driver's 8-GPU run
takes the same code path on RCCL (there with the native communicator and a captured step)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(150)   # rank 0 tunes, rank 1 takes its variant table (ssseg.tune): no longer minutes per rank
def test_bench_two_ranks_gloo_one_gpu(hip_device):
    env = dict(os.environ, SSSEG_BENCH_BACKEND='gloo', HSA_ENABLE_IPC_MODE_LEGACY='0')
    env.pop('WORLD_SIZE', None)
    steps, batch = 2, 2
    p = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '2', '--steps', str(steps), '--warmup',
                        '1', '--batch', str(batch), '--size', '64', '--no-cpu-baseline', '--no-fp32'],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, p.stdout[-2000:]       # rank 0 only
    r = json.loads(lines[0])
    assert r['n_gpus'] == 2 and r['config']['parallelism'] == 'dp2' and r['scaling'] == 'weak'
    assert r['config']['global_batch'] == 2 * batch
    # value = all ranks' images / the MAX-over-ranks elapsed time of exactly `steps` steps
    elapsed = r['ms_per_step'] * steps / 1e3
    assert abs(r['value'] - 2 * batch * steps / elapsed) <= 1e-3 * r['value'] + 1e-3
    assert r['execution'].startswith('eager')
    assert r['liveness']['losses_finite']
    # every rank holds rank 0's conv variant table (ssseg.tune.sync; bench.py raises on a mismatch before the timed steps)
    digests = r['conv_variant_table']['digest_per_rank']
    assert len(digests) == 2 and digests[0] == digests[1] and r['conv_variant_table']['rows'] > 0
    assert r['collectives']['transport'] == 'c10d' and r['collectives']['backend'] == 'gloo'
    assert 'backend gloo' in p.stderr and p.stderr.count('process group: world 2') == 2
