import os, sys, numpy as np
sys.path.insert(0, '.')
import rvcp_amd
sc = rvcp_amd.Scene.default()
out = {}
for size, spp in [(1024, 30), (384, 10), (200, 7)]:
    with rvcp_amd.RayTracer(spp=spp) as rt:
        rt.upload_scene(sc)
        rgba, lin = rt.render(size, size, 123.0, want_linear=True)
    np.save(f"gpurun_out/spec_{os.environ.get('TAG','x')}_{size}.npy", lin)
    print(size, float(lin.sum()), flush=True)
