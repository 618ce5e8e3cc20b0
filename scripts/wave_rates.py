import json, sys
sys.path[:0] = ['.', 'radiative-transfer_amd']
import bench, rtsn
pdir = bench.REPO / 'tests' / 'golden' / 'prm'
for name in bench.REFERENCE_CONFIGS:
    ph = rtsn.ParameterHandler(pdir / name, table_dir=str(pdir) + '/')
    q = ph.params
    g = bench.gpu_rate(q, q['ts_method'], 1000)
    print(json.dumps(dict(config=name, rep=int(sys.argv[1]), **g)), flush=True)
