"""The N > 1 bench path on real ranks: bench.py --gpus 2 through
torch.distributed.run, one process per GPU, owner-computes (exchange 2) and peer-write
(exchange 1) DB shards on 2 x 256^2 jobs (every level pruned and sharded) and 2 x 1024^2 jobs
(cfg3: the 1024^2 level), plus the one-job strong run.  bench.py itself compares every rank's
sharded job bit for bit with the same job run alone on that GPU (shard_parity) and the one-job
sharded run with rank 0's single-GPU run (strong_parity) and exits 3 on a mismatch.

Needs >= 2 visible GPUs (skipped otherwise).  IA_TEST_SHARE_GPU=1 rehearses it on one GPU (the
ranks share the device on disjoint CU halves, gloo for the host collectives; bench.py's
IA_BENCH_SHARE_GPU) - the driver never sets it.  The child processes are started before this
process touches the GPU state they use: device_count() does not initialise HIP on this image."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _ranks_available():
    import torch
    if torch.cuda.device_count() >= 2:
        return 'gpus'
    if os.environ.get('IA_TEST_SHARE_GPU') == '1' and torch.cuda.device_count() >= 1:
        return 'share'
    return None


@pytest.mark.parametrize('config,exchange', [('s256', 'owner'), ('s256', 'peer'), ('cfg3', 'owner'), ('cfg3', 'peer')])
def test_two_ranks_bit_exact_to_single_gpu(config, exchange, tmp_path):
    mode = _ranks_available()
    if mode is None:
        pytest.skip('needs 2 GPUs (or IA_TEST_SHARE_GPU=1 for the one-GPU rehearsal)')
    env = dict(os.environ)
    if mode == 'share':
        env.update(IA_BENCH_SHARE_GPU='1', IA_BENCH_BACKEND='gloo')
    port = 29600 + 7 * ['s256', 'cfg3'].index(config) + ['owner', 'peer'].index(exchange)
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2',
           '--master-addr', '127.0.0.1', '--master-port', str(port), os.path.join(ROOT, 'bench.py'),
           '--gpus', '2', '--steps', '1', '--warmup', '1', '--no-cpu-baseline', '--no-replicas-extra',
           '--config', config, '--exchange', exchange]
    if config == 's256':
        cmd += ['--prune-min-rows', '1']   # every level pruned; the 128^2 and 256^2 levels shard 2 ways
    r = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=400)
    (tmp_path / 'err.txt').write_bytes(r.stderr)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    line = json.loads(r.stdout.decode().strip().splitlines()[-1])
    assert 'shard_error' not in line['config'], line['config'].get('shard_error')
    assert line['shard_parity'] is True
    assert line['strong_parity'] is True and line['value_strong'] > 0
    # the headline is BASELINE config 3 as named: ONE job, its DB sharded over the ranks (strong
    # scaling); the N-job weak reading rides along as value_weak
    assert line['value'] == line['value_strong'] and line['scaling'] == 'strong'
    assert line['config']['jobs_per_step'] == 1 and line['config']['parallelism'].endswith('_jobs1')
    assert line['value_weak'] > 0 and line['config']['weak']['scaling'] == 'weak'
    assert line['stats']['bound_violations'] == 0 and line['stats']['kappa_ambiguous'] == 0


def _bench(args, env, port=None, nproc=1, timeout=600):
    if nproc > 1:
        cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', str(nproc),
               '--master-addr', '127.0.0.1', '--master-port', str(port), os.path.join(ROOT, 'bench.py')]
    else:
        cmd = [sys.executable, os.path.join(ROOT, 'bench.py')]
    r = subprocess.run(cmd + args, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=timeout)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    return json.loads(r.stdout.decode().strip().splitlines()[-1])


def test_cfg5_sweep_two_ranks_equal_one_gpu(tmp_path):
    """BASELINE config 5 on two ranks: the 64-job sweep split job j -> rank
    j mod 2 with no collective on the data path.  Every job's B', s, im (every level; bench.py
    job_digests, one sha1 per job, gathered over the ranks as host objects) must equal the same
    job of a one-GPU run of the whole sweep, and each rank's timed run must equal its own one-stream
    rerun (parity)."""
    mode = _ranks_available()
    if mode is None:
        pytest.skip('needs 2 GPUs (or IA_TEST_SHARE_GPU=1 for the one-GPU rehearsal)')
    env = dict(os.environ)
    common = ['--steps', '1', '--warmup', '1', '--no-cpu-baseline', '--no-replicas-extra', '--config', 'cfg5']
    one = _bench(['--gpus', '1'] + common, env)
    if mode == 'share':
        env.update(IA_BENCH_SHARE_GPU='1', IA_BENCH_BACKEND='gloo')
    two = _bench(['--gpus', '2'] + common, env, port=29641, nproc=2)
    assert one['parity'] is True and two['parity'] is True
    assert len(one['job_digests']) == 64 and two['job_digests'] == one['job_digests']
    assert two['n_gpus'] == 2 and two['config']['parallelism'] == 'jobs2'
    assert two['stats']['bound_violations'] == 0 and two['stats']['kappa_ambiguous'] == 0
