"""Reproduce: a chain test after four-attribute wide-kernel runs in the same process."""
import os, sys, json
sys.path.insert(0, 'mpi-model_amd'); sys.path.insert(0, 'oracle')
import numpy as np
import mpimodel as mm
mm.lib()
import oracle as O
C5 = [(2, 0, 1, 0.05), (2, 1, 2, 0.03), (2, 2, 3, 0.02), (2, 3, 0, 0.01),
      (1, 0, 0, 0.1), (1, 1, 1, 0.1), (1, 2, 2, 0.05), (1, 3, 3, 0.2)]


def wide4(H, W, env, steps=21, red=1):
    os.environ.update({k: str(v) for k, v in env.items()})
    e = mm.Engine(H, W, n_attr=4)
    for k in env: os.environ.pop(k)
    for a in range(4):
        e.fill_random(a, seed=O.SEED + a)
    for kind, a, b, r in C5:
        (e.add_diffuse(a, r) if kind == 1 else e.add_transfer(a, b, r))
    e.run(steps, red)
    got = [e.download(a) for a in range(4)]
    e.close()
    fields = [O.fill_random(H, W, seed=O.SEED + a) for a in range(4)]
    want = O.program_step(fields, C5, steps=steps)
    return all(np.array_equal(got[a], want[a]) for a in range(4))


def chain(H=64, W=300, G=2, k=10, mode=0):
    os.environ.update({"MM_STEPS_PER_PASS": str(k), "MM_WIDE": "0"})
    engines = []
    for g in range(G):
        x0, h = mm.partition_rows(H, G, g)
        engines.append(mm.Engine(H, W, x0, h, rank=g, nranks=G, halo_mode=mm.MM_HALO_HOST))
    for kk in ("MM_STEPS_PER_PASS", "MM_WIDE"): os.environ.pop(kk)
    for e in engines:
        e.fill_random(0); e.add_diffuse(0, 0.3)
    steps = 2 * engines[0].info()["halo_depth"] + 1
    plan = engines[0].pass_plan(steps)
    for kk in plan:
        halos = [e.halo_export(kk) for e in engines]
        for g, e in enumerate(engines):
            e.halo_import(halos[g-1][1] if g > 0 else None, halos[g+1][0] if g < G-1 else None, nrows=kk)
        if mode == 1:
            mm.device_synchronize(0)
        for e in engines:
            e.run(kk)
            if mode == 2:
                e.synchronize()
                mm.device_synchronize(0)
    got = np.vstack([e.download() for e in engines])
    for e in engines: e.close()
    want = O.field_step(O.fill_random(H, W), 0.3, steps=steps)
    bad = np.nonzero((got != want).any(axis=1))[0]
    return {"plan": plan, "nbad": int(len(bad)), "bad": bad.tolist()[:12]}




def single(H=64, W=300, k=10, steps=21, env_extra=None):
    env = {"MM_STEPS_PER_PASS": str(k), "MM_WIDE": "0"}
    env.update(env_extra or {})
    os.environ.update(env)
    e = mm.Engine(H, W)
    for kk in env: os.environ.pop(kk)
    e.fill_random(0); e.add_diffuse(0, 0.3)
    plan = e.pass_plan(steps)
    e.run(steps)
    got = e.download()
    e.close()
    want = O.field_step(O.fill_random(H, W), 0.3, steps=steps)
    bad = np.nonzero((got != want).any(axis=1))[0]
    return {"plan": plan, "nbad": int(len(bad)), "bad": bad.tolist()[:12]}


def chain1(H=64, W=300, G=2, k=10, plan=(7,)):
    os.environ.update({"MM_STEPS_PER_PASS": str(k), "MM_WIDE": "0"})
    engines = []
    for g in range(G):
        x0, h = mm.partition_rows(H, G, g)
        engines.append(mm.Engine(H, W, x0, h, rank=g, nranks=G, halo_mode=mm.MM_HALO_HOST))
    for kk in ("MM_STEPS_PER_PASS", "MM_WIDE"): os.environ.pop(kk)
    for e in engines:
        e.fill_random(0); e.add_diffuse(0, 0.3)
    init = np.vstack([e.download() for e in engines])
    ok_init = bool(np.array_equal(init, O.fill_random(H, W)))
    for kk in plan:
        halos = [e.halo_export(kk) for e in engines]
        for g, e in enumerate(engines):
            e.halo_import(halos[g-1][1] if g > 0 else None, halos[g+1][0] if g < G-1 else None, nrows=kk)
        for e in engines:
            e.run(kk)
    got = np.vstack([e.download() for e in engines])
    ghost = [e.read_rows(-kk, kk) for e in engines]
    for e in engines: e.close()
    want = O.field_step(O.fill_random(H, W), 0.3, steps=sum(plan))
    bad = np.nonzero((got != want).any(axis=1))[0]
    return {"ok_init": ok_init, "nbad": int(len(bad)), "bad": bad.tolist()[:40],
            "ghost_e1_top_vs_e0_bottom": None}


for rep in range(2):
    wide4(257, 512, {"MM_WIDE": 0}, steps=2)
    print(json.dumps({"single": single()}), flush=True)
    wide4(257, 512, {"MM_WIDE": 0}, steps=2)
    print(json.dumps({"chain [7]": chain1(plan=(7,))}), flush=True)
    wide4(257, 512, {"MM_WIDE": 0}, steps=2)
    print(json.dumps({"chain [1]": chain1(plan=(1,))}), flush=True)
    wide4(257, 512, {"MM_WIDE": 0}, steps=2)
    print(json.dumps({"chain [7] K7": chain1(k=7, plan=(7,))}), flush=True)
sys.exit(0)
print(json.dumps({"chain first": chain()}), flush=True)
for rep in range(3):
    for mode in (0, 1, 2):
        wide4(257, 512, {"MM_WIDE": 0}, steps=2)
        r = chain(mode=mode)
        print(json.dumps({"rep": rep, "mode": mode, "nbad": r["nbad"], "bad": r["bad"]}), flush=True)
for mode in (0, 1, 2):
    wide4(257, 512, {"MM_WIDE": 0}, steps=2)
    r = chain(H=64, W=300, G=2, k=7, mode=mode)
    print(json.dumps({"k7": True, "mode": mode, "nbad": r["nbad"]}), flush=True)
    wide4(257, 512, {"MM_WIDE": 0}, steps=2)
    r = chain(H=300, W=700, G=2, k=10, mode=mode)
    print(json.dumps({"300x700": True, "mode": mode, "nbad": r["nbad"], "plan": r["plan"]}), flush=True)
sys.exit(0)
