"""The distinct-proof pool of BASELINE config 4 — TEST DATA GENERATOR ONLY.

Config 4 is 4,096 transaction proofs with log2 padded heights drawn from the
ProofCollection member mix {16, 10, 11, 12, 12, 11, 9, 9}.  Its proofs come from a pool of 256
distinct accepting proofs, in the mix's proportions (heights 9 / 10 / 11 / 12 / 16: 64 / 32 / 64 /
64 / 32), each with its own claim (digest, input and output of varying lengths) and prover seed:

  * the first proof of each height is the committed full synthetic proof of tests/golden/c3_pool.npz
    (oracle/stark_prover_fast.py: every column a low-degree polynomial);
  * the other 251 come from the sparse prover (oracle/stark_prover_sparse.py: one non-constant
    column, non-zero FRI in every round), cheap enough to make on the machine that runs them.

Every proof is verified by both oracle restatements (oracle/stark_ref.py, oracle/stark_oracle.c)
before the pool is written (all accept), and the Python oracle's Fiat-Shamir transcript of each
(every squeezed sample, the FRI indices) is kept with it for the GPU transcript comparison.  The pool is built in a child process (a pool of forked workers, none of which has touched a
GPU) and cached under the system temp directory, keyed by the generator sources and the c3 pool, so
the bench and the GPU tests of one machine build it once.  Used by bench.py (config 4) and
tests/test_gpu_config4.py; never by the product.

Usage: python oracle/pool4.py --out PATH [--workers N]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
C3_POOL = os.path.join(ROOT, "tests", "golden", "c3_pool.npz")
HEIGHT_COUNTS = {9: 64, 10: 32, 11: 64, 12: 64, 16: 32}
SEED = 0xC4


def _claim(h: int, j: int):
    """Distinct claim per (height, j): digest, input and output lengths vary with j."""
    digest = [h, j, SEED, (j * 7919) % 65521, 0x5EED]
    inp = [(h * 1000 + j * 13 + k) for k in range(j % 7)]
    out = [(j * 31 + k) for k in range(j % 3)]
    return digest, 0, inp, out


def _prove_one(task):
    """One pool entry in a worker process: the proof (j = 0: the committed full proof of that height;
    else a sparse-prover proof) and the oracle verifier's transcript of it (every squeezed sample,
    the FRI indices)."""
    h, j = task
    sys.path.insert(0, HERE)
    import stark_prover_fast as F
    import stark_prover_sparse as SP
    import stark_ref as S
    import tip5_ref as T
    F.THREADS = 1  # one proof per worker process
    T.use_c_backend()
    params = S.StarkParams()
    air, recipe = S.synth_air(params, seed=1)
    if j == 0:
        z = np.load(C3_POOL)
        c = json.loads(bytes(z["meta"]).decode())["claims"][str(h)]
        claim = (c["digest"], c["version"], c["input"], c["output"])
        proof = z[f"proof_{h}"]
        assert [int(w) for w in z["air"]] == air.to_words(), "c3 pool AIR is not synth_air(seed=1)"
    else:
        claim = _claim(h, j)
        proof, _, _ = SP.prove(params, air, recipe, claim, h, seed=(SEED << 16) + (h << 8) + j)
    proof = np.asarray(proof, dtype=np.uint64)
    tr = {}
    if not S.verify(params, air, claim, [int(w) for w in proof], tr):
        raise RuntimeError(f"pool proof ({h}, {j}) rejected by the Python oracle")
    samples = np.array([x for tag, vals in tr["sponge_samples"] if tag != "fri_indices" for x in vals],
                       dtype=np.uint64)
    indices = np.array([v for tag, vals in tr["sponge_samples"] if tag == "fri_indices" for v in vals],
                       dtype=np.uint64)
    return h, j, claim, proof, samples, indices


def _main_rows_range(proof, params):
    import stark_ref as S
    items = S.decode_proof([int(w) for w in proof], params)
    pos = 2
    for k, _ in items:
        ln = int(proof[pos])
        if k == S.MAIN_ROWS:
            return pos + 1, pos + 1 + ln
        pos += 1 + ln
    raise ValueError("no MainRows item")


def build(out_path: str, workers: int) -> None:
    sys.path.insert(0, HERE)
    import coracle as C
    import stark_ref as S
    from concurrent.futures import ProcessPoolExecutor
    t0 = time.time()
    params = S.StarkParams()
    air = np.load(C3_POOL)["air"]
    entries = []  # (height, j, claim, proof, kind, samples, indices)
    tasks = [(h, j) for h in sorted(HEIGHT_COUNTS, reverse=True) for j in range(HEIGHT_COUNTS[h])]
    with ProcessPoolExecutor(max_workers=workers) as ex:
        for h, j, claim, proof, smp, idx in ex.map(_prove_one, tasks, chunksize=1):
            entries.append((h, j, claim, proof, "full" if j == 0 else "sparse", smp, idx))
    entries.sort(key=lambda e: (e[0], e[1]))
    claims = [e[2] for e in entries]
    proofs = [e[3] for e in entries]
    ok = C.stark_verify_batch([int(w) for w in air], params, claims, proofs, threads=workers)
    if not all(bool(x) for x in ok):
        raise RuntimeError(f"pool proofs rejected by the oracle: {[i for i, x in enumerate(ok) if not x]}")
    offs = np.zeros(len(proofs) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(p) for p in proofs])
    soffs = np.zeros(len(proofs) + 1, dtype=np.uint64)
    soffs[1:] = np.cumsum([e[5].shape[0] for e in entries])
    ioffs = np.zeros(len(proofs) + 1, dtype=np.uint64)
    ioffs[1:] = np.cumsum([e[6].shape[0] for e in entries])
    info = {"heights": [e[0] for e in entries], "j": [e[1] for e in entries], "kind": [e[4] for e in entries],
            "claims": [{"digest": c[0], "version": c[1], "input": c[2], "output": c[3]} for c in claims],
            "main_rows": [list(_main_rows_range(p, params)) for p in proofs],
            "build_s": time.time() - t0, "workers": workers}
    tmp = out_path + f".tmp{os.getpid()}.npz"
    np.savez(tmp, air=air, words=np.concatenate(proofs), offsets=offs,
             samples=np.concatenate([e[5] for e in entries]), sample_offsets=soffs,
             indices=np.concatenate([e[6] for e in entries]), index_offsets=ioffs,
             meta=np.frombuffer(json.dumps(info).encode(), dtype=np.uint8))
    os.replace(tmp, out_path)


def _key() -> str:
    h = hashlib.sha256()
    for f in ("pool4.py", "stark_prover_sparse.py", "stark_prover_fast.py", "stark_prover_const.py",
              "stark_ref.py", "vec_oracle.c", "tip5_oracle.c", "stark_oracle.c"):
        h.update(open(os.path.join(HERE, f), "rb").read())
    h.update(open(C3_POOL, "rb").read())
    return h.hexdigest()[:16]


def load(workers: int | None = None, timeout_s: float = 1800.0) -> dict:
    """The pool (building it once per machine): {"air", "proofs", "claims", "heights", "main_rows",
    "kind"}.  The first caller builds it in a child process; concurrent callers (the ranks of one
    node) wait for the file."""
    workers = workers or min(16, os.cpu_count() or 1)
    path = os.path.join(tempfile.gettempdir(), f"nhip_pool4_{_key()}.npz")
    lock = path + ".lock"
    if not os.path.exists(path):
        try:
            fd = os.open(lock, os.O_CREAT | os.O_EXCL | os.O_WRONLY)
            os.close(fd)
            try:
                subprocess.run([sys.executable, os.path.abspath(__file__), "--out", path, "--workers", str(workers)],
                               check=True)
            finally:
                os.unlink(lock)
        except FileExistsError:
            t = time.time()
            while not os.path.exists(path):
                if time.time() - t > timeout_s or not os.path.exists(lock):
                    if os.path.exists(path):
                        break
                    raise RuntimeError("config-4 pool: the building process did not finish")
                time.sleep(0.5)
    z = np.load(path)
    info = json.loads(bytes(z["meta"]).decode())
    words, offs = z["words"], z["offsets"]
    proofs = [words[int(offs[i]):int(offs[i + 1])] for i in range(len(offs) - 1)]
    claims = [(c["digest"], c["version"], c["input"], c["output"]) for c in info["claims"]]
    smp, so = z["samples"], z["sample_offsets"]
    idx, io = z["indices"], z["index_offsets"]
    transcripts = [([tuple(int(c) for c in x) for x in smp[int(so[i]):int(so[i + 1])]],
                    [int(v) for v in idx[int(io[i]):int(io[i + 1])]]) for i in range(len(proofs))]
    return {"air": z["air"], "proofs": proofs, "claims": claims, "heights": info["heights"],
            "main_rows": info["main_rows"], "kind": info["kind"], "transcripts": transcripts,
            "build_s": info.get("build_s"), "path": path}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--workers", type=int, default=min(16, os.cpu_count() or 1))
    a = ap.parse_args()
    build(a.out, a.workers)
