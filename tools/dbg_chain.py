import os, sys, json
sys.path.insert(0, 'mpi-model_amd'); sys.path.insert(0, 'oracle')
import numpy as np
import mpimodel as mm
mm.lib()
import oracle as O
H, W, G = 64, 300, 2
for env in ({"MM_STEPS_PER_PASS": "10", "MM_WIDE": "0"}, {"MM_WIDE": "0"}):
    os.environ.update(env)
    for plan in ([7, 7, 7], [10, 10, 1], [7], [10], [3, 4]):
        engines = []
        for g in range(G):
            x0, h = mm.partition_rows(H, G, g)
            engines.append(mm.Engine(H, W, x0, h, rank=g, nranks=G, halo_mode=mm.MM_HALO_HOST))
        for e in engines:
            e.fill_random(0); e.add_diffuse(0, 0.3)
        for k in plan:
            halos = [e.halo_export(k) for e in engines]
            for g, e in enumerate(engines):
                e.halo_import(halos[g-1][1] if g > 0 else None, halos[g+1][0] if g < G-1 else None, nrows=k)
            for e in engines:
                e.run(k)
        got = np.vstack([e.download() for e in engines])
        want = O.field_step(O.fill_random(H, W), 0.3, steps=sum(plan))
        bad = np.nonzero((got != want).any(axis=1))[0]
        print(json.dumps({"env": env, "plan": plan, "info_depth": engines[0].info()["halo_depth"],
                          "bad_rows": bad.tolist()[:40], "nbad": int(len(bad)),
                          "zero_rows": np.nonzero((got == 0).all(axis=1))[0].tolist()[:20]}), flush=True)
        for e in engines: e.close()
    for k in env: os.environ.pop(k)
