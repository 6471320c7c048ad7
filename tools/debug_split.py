import ctypes, sys, os
sys.path.insert(0, "tests")
import numpy as np
import helpers
rt580 = helpers.rt580(); lib = rt580.load()
import torch
d = helpers.rt580_dist()
scene, w, h, depth, ao = "simpleSphereScene.json", 97, 61, 4, 64
rt = rt580.Raytracer(w, h, helpers.ASSETS_ROOT)
rt.LoadSceneJSON(scene); rt.set_depth(depth); rt.set_ao(ao, True); rt.Render("")
full = rt.framebuffer()
params = rt.render_params()
dev = torch.device("cuda", 0)
rt580.check(lib.rt_gpu_set_stream(ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)), "stream")
for world in (1, 2):
    backend = d.GpuRows(rt580, params, torch, dev)
    n_max = d.n_max_rows(h, world)
    counts = [backend.count(r, world).clone() for r in range(world)]
    fc = torch.stack(counts, dim=1).reshape(-1)[:h].to(torch.int64)
    base = torch.cumsum(fc, 0) - fc
    print("world", world, "counts", fc.tolist()[:40])
    for r in range(world):
        backend.count(r, world)
        lb = torch.zeros(n_max, dtype=torch.int64, device=dev)
        mine = base[r::world]; lb[:mine.numel()] = mine
        tile = backend.shade(r, world, lb).view(n_max, w, 3).cpu().numpy()
        rows = list(range(r, h, world))
        bad = [y for k, y in enumerate(rows) if not np.array_equal(tile[k], full[y])]
        print(" rank", r, "bad rows", bad[:8], "bases", lb.tolist()[:12])
        if bad:
            k = rows.index(bad[0]); y = bad[0]
            diff = np.argwhere((tile[k] != full[y]).any(axis=1)).ravel()
            print("   row", y, "first diff x", diff[:10].tolist(), tile[k][diff[0]], full[y][diff[0]])
