#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the reference itself.

TEST INFRASTRUCTURE. Runs only in the build container, where /root/reference
exists: `make -C oracle ref` compiles the reference (oracle/_ref/), then this
script runs it under MPICH `mpirun -np NWORKERS+1` (the only working reference
layout) and records, per case, every cell whose final value
differs from the reference's init value 1.0 (Model.hpp:155), as exact hex floats.

Cases stay inside the reference's valid oracle domain:
source row == PROC_DIMX-1 (last row of worker 1's slab), interior column.

Three fixture kinds:
  point_<geom>_<n>.json  exact grids from oracle/_ref/ref_<geom> (our driver over
                         the unmodified reference headers, hex-float dump)
  c1_default_text.json   the reference's own Main.cpp build: sha256 + the
                         non-trivial lines of every comm_rank%d.txt it writes at
                         default ostream precision (Model.hpp:246-257) -- the
                         byte-level format the drop-in writer must reproduce.
  wire_<model>_<geom>_<n>.json  every MPI_Send the reference makes (oracle/_ref/wire_*:
                         oracle/ref_wire_harness.cpp interposes MPI_Send over the unmodified
                         reference headers): the 23-char partition / flow descriptors of
                         Model (src/Model.hpp:70-86) and ModelRectangular's 2-D blocks
                         (src/ModelRectangular.hpp:69-92), halo scalars, sums, file names.
"""
import hashlib
import json
import math
import os
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_DIR = os.path.join(REPO, "oracle", "_ref")
MPIRUN = os.environ.get("MPIRUN", "/opt/conda/bin/mpirun")

# (geometry DIMX_DIMY_NWORKERS, src_x, src_y, captured value, rate)
CASES = [
    ("100_100_5", 19, 3, "2.2", "0.1"),            # Main.cpp:33 default
    ("100_100_5", 19, 50, "1.2345678901234567", "0.123456789"),
    ("100_100_5", 19, 98, "7.5", "0.9"),
    ("40_64_4", 9, 17, "3.5", "0.25"),              # SURVEY.md section 4 case
    ("40_64_4", 9, 1, "0.3", "0.7"),
    ("60_30_3", 19, 28, "1.7", "0.3"),
    ("24_16_2", 11, 1, "5.0", "0.05"),
    ("24_16_2", 11, 14, "3.0", "1.0"),
    ("64_128_8", 7, 64, "2.0", "0.5"),
    ("36_50_6", 5, 25, "9.99", "0.333"),
]


def run_ref(binary, np_, args, timeout=60):
    work = tempfile.mkdtemp(prefix="mmref_")
    run = os.path.join(work, "run")
    out = os.path.join(work, "output")
    os.makedirs(run)
    os.makedirs(out)
    proc = subprocess.run([MPIRUN, "-np", str(np_), binary] + list(args), cwd=run,
                          capture_output=True, text=True, timeout=timeout)
    if proc.returncode != 0:
        raise RuntimeError(f"{binary} failed: {proc.stderr}")
    files = {}
    for name in sorted(os.listdir(out)):
        with open(os.path.join(out, name), "rb") as f:
            files[name] = f.read()
    shutil.rmtree(work)
    return proc.stdout, files


def point_case(geom, sx, sy, value, rate):
    dimx, dimy, nw = (int(t) for t in geom.split("_"))
    stdout, files = run_ref(os.path.join(REF_DIR, f"ref_{geom}"), nw + 1,
                            [str(sx), str(sy), value, rate])
    cells = {}
    for k in range(1, nw + 1):
        text = files[f"comm_rank{k}.txt"].decode()
        for line in text.splitlines():
            x, y, v = line.split("\t")
            cells[(int(x), int(y))] = float.fromhex(v)
    assert len(cells) == dimx * dimy, (geom, len(cells))
    changed = sorted((x, y, v.hex()) for (x, y), v in cells.items() if v != 1.0)
    total = math.fsum(cells.values())
    return {
        "kind": "point",
        "dimx": dimx, "dimy": dimy, "nworkers": nw, "np": nw + 1,
        "src_x": sx, "src_y": sy,
        "value": value, "value_hex": float(value).hex(),
        "rate": rate, "rate_hex": float(rate).hex(),
        "init_value_hex": (1.0).hex(),
        "changed": [[x, y, h] for x, y, h in changed],
        "sum_fsum_hex": total.hex(),
        "reference_stdout": stdout,
        "generator": "oracle/_ref/ref_%s (oracle/ref_harness.cpp over /root/reference/src)" % geom,
    }


# Sources OUTSIDE the valid domain that the reference still completes (SURVEY.md section
# 0: other sources crash or hang): with one worker, or in the last of two workers' slabs,
# it changes no cell (src/Model.hpp:189-216). Pins the strict-reference point mode.
STRICT_CASES = [
    ("24_16_1", 11, 7, "2.0", "0.5"),    # interior, not the slab's last row
    ("24_16_1", 23, 7, "2.0", "0.5"),    # the slab's last row = the grid's: 5 neighbours
    ("24_16_1", 0, 5, "2.0", "0.5"),     # top edge
    ("24_16_1", 23, 15, "2.0", "0.5"),   # corner: 3 neighbours
    ("30_20_1", 14, 9, "1.5", "0.25"),
    ("30_20_1", 29, 10, "1.5", "0.25"),
    ("24_16_2", 15, 7, "2.0", "0.5"),    # last worker, interior, not its last row
    ("24_16_2", 20, 8, "3.0", "0.1"),
    ("24_16_2", 23, 0, "2.0", "0.5"),
]

# (model, geometry, np, src_x, src_y, value, rate, space h/w or None)
WIRE_CASES = [
    ("row", "100_100_5", 6, 19, 3, "2.2", "0.1", None),       # Main.cpp:33 default
    ("row", "40_64_4", 5, 9, 17, "3.5", "0.25", None),
    ("rect", "20_60_2_3", 7, 18, 19, "2.2", "0.1", None),     # Main.cpp:37-47 (commented)
    ("rect", "24_60_3_2", 7, 5, 7, "1.5", "0.3", None),
    ("rect", "20_61_2_3", 7, 3, 4, "1.0", "0.5", None),       # DIMY_REC % COLUMNS_REC != 0
    ("rect", "30_40_3_4", 13, 7, 11, "2.0", "0.2", (12, 9)),
]


def wire_case(model, geom, np_, sx, sy, value, rate, space):
    binary = os.path.join(REF_DIR, f"wire_{model}_{geom}")
    args = [model, str(sx), str(sy), value, rate] + ([str(space[0]), str(space[1])] if space else [])
    work = tempfile.mkdtemp(prefix="mmwire_")
    os.makedirs(os.path.join(work, "run"))
    os.makedirs(os.path.join(work, "output"))
    proc = subprocess.run([MPIRUN, "-np", str(np_), binary] + args, cwd=os.path.join(work, "run"),
                          capture_output=True, text=True, timeout=60)
    shutil.rmtree(work)
    if proc.returncode != 0:
        raise RuntimeError(f"{binary} failed: {proc.stderr[-2000:]}")
    sends = {}
    for ln in proc.stderr.splitlines():
        if not ln.startswith("MPISEND "):
            continue
        f = dict(kv.split("=", 1) for kv in ln[8:].split(" ", 5))
        sends.setdefault(int(f["src"]), []).append(
            [int(f["dest"]), int(f["tag"]), f["type"], int(f["count"]), f["data"]])
    dims = [int(t) for t in geom.split("_")]
    fx = {"kind": "wire", "model": model, "np": np_, "src_x": sx, "src_y": sy,
          "value": value, "rate": rate,
          "sends_by_rank": {str(k): v for k, v in sorted(sends.items())},
          "reference_stdout_lines": sorted(proc.stdout.splitlines()),
          "generator": f"oracle/_ref/wire_{model}_{geom} (oracle/ref_wire_harness.cpp over "
                       f"/root/reference/src)"}
    if model == "row":
        fx.update(dimx=dims[0], dimy=dims[1], nworkers=dims[2])
    else:
        fx.update(dimx_rec=dims[0], dimy_rec=dims[1], lines_rec=dims[2], columns_rec=dims[3],
                  space=list(space) if space else [dims[0] // dims[2], dims[1] // dims[3]])
    return fx


def c1_text_case():
    stdout, files = run_ref(os.path.join(REF_DIR, "ref_main_default"), 6, [])
    ranks = {}
    merged = [v for k, v in sorted(files.items()) if k.startswith("comm_rank")]
    for name, data in sorted(files.items()):
        if not name.startswith("comm_rank"):
            continue
        lines = data.decode().splitlines()
        ranks[name] = {
            "sha256": hashlib.sha256(data).hexdigest(),
            "n_lines": len(lines),
            "lines_not_1": [ln for ln in lines if not ln.endswith("\t1")],
            "first_line": lines[0], "last_line": lines[-1],
        }
    merged_names = [k for k in files if k.startswith("output ")]
    merged_sha = hashlib.sha256(files[merged_names[0]]).hexdigest() if merged_names else None
    return {
        "kind": "c1_text",
        "dimx": 100, "dimy": 100, "nworkers": 5, "np": 6,
        "src_x": 19, "src_y": 3, "value": "2.2", "rate": "0.1",
        "rank_files": ranks,
        "concat_sha256": hashlib.sha256(b"".join(merged)).hexdigest(),
        "merged_file_sha256": merged_sha,
        "reference_stdout": stdout,
        "generator": "oracle/_ref/ref_main_default (/root/reference/src/Main.cpp unchanged)",
    }


def main():
    if not os.path.isdir("/root/reference"):
        sys.exit("make_golden.py runs only where /root/reference exists")
    subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "ref"], check=True,
                   capture_output=True)
    index = []
    for i, (geom, sx, sy, value, rate) in enumerate(CASES):
        fx = point_case(geom, sx, sy, value, rate)
        name = f"point_{geom}_{i}.json"
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(fx, f, indent=1)
        index.append(name)
        print(name, len(fx["changed"]), "cells changed")
    for i, (geom, sx, sy, value, rate) in enumerate(STRICT_CASES):
        fx = point_case(geom, sx, sy, value, rate)
        fx["kind"] = "strict"
        name = f"strict_{geom}_{i}.json"
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(fx, f, indent=1)
        index.append(name)
        print(name, len(fx["changed"]), "cells changed")
    for i, case in enumerate(WIRE_CASES):
        fx = wire_case(*case)
        name = f"wire_{case[0]}_{case[1]}_{i}.json"
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(fx, f, indent=1)
        index.append(name)
        print(name, sum(len(v) for v in fx["sends_by_rank"].values()), "messages")
    fx = c1_text_case()
    with open(os.path.join(HERE, "c1_default_text.json"), "w") as f:
        json.dump(fx, f, indent=1)
    index.append("c1_default_text.json")
    with open(os.path.join(HERE, "index.json"), "w") as f:
        json.dump(index, f, indent=1)


if __name__ == "__main__":
    main()
