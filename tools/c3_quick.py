import os, sys, time, json, hashlib
sys.path.insert(0, os.getcwd())
import torch
import ccphylo_amd as cg
from tools.synth import euclid_shard_dev
n = 200000
dev = cg.Device(0)
D = euclid_shard_dev(torch, n, 0, 1, dtype=torch.float32)
host = D.cpu()
for st_ in sys.argv[1:]:
    env = dict(kv.split("=", 1) for kv in st_.split())
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    D.copy_(host); torch.cuda.synchronize()
    t0 = time.perf_counter()
    j, fn, fd, st = dev.tree_dev(D.data_ptr(), n, etype=4, method=cg.CCG_TREE_DNJ, exact=True, max_joins=20000)
    dt = time.perf_counter() - t0
    print(json.dumps({"settings": st_ or "defaults", "joins": len(j), "s": round(dt, 3), "sha": hashlib.sha256(j.tobytes()).hexdigest()[:16], "rows": st[0], "cells": st[1]}), flush=True)
    for k, v in old.items():
        if v is None: os.environ.pop(k, None)
        else: os.environ[k] = v
