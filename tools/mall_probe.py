import json, os, sys
sys.path.insert(0, '/root/repo') if os.path.exists('/root/repo') else None
sys.path.insert(0, os.environ.get('GRAFT_REPO_ROOT', '.'))
import ia_amd
from ia_amd import _native
ctx = _native.Context(0)
ctx.set_option('k3_variant', 1)
for n in (262144, 524288, 655360, 786432, 917504, 1048576):
    for M in (32, 342):
        us = ctx.k3_microbench(n, M, 30)
        print(json.dumps({'n_rows': n, 'db_MiB': n * 256 / 2**20, 'M': M, 'us': round(us, 1),
                          'GBps': round(n * 256 / (us * 1e-6) / 1e9)}), flush=True)
