#!/bin/bash
# The oracle's volumetric path (trackGrid with 16^3-voxel majorant cells, the round-3 fault
# configuration of the kernels) under AddressSanitizer on the host: a guided smoke render at reduced
# resolution with records, splat and refit.  CPU only.
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p /tmp/orc_asan
g++ -O1 -g -std=c++17 -fPIC -pthread -ffp-contract=off -fsanitize=address -fno-omit-frame-pointer \
    -DORC_MAJORANT_CELL=${CELL:-16} -shared -o /tmp/orc_asan/liboracle.so oracle/oracle.cpp
ASAN_OPTIONS=detect_leaks=0 LD_PRELOAD=$(g++ -print-file-name=libasan.so) ORACLE_LIB=/tmp/orc_asan/liboracle.so python - <<'PY'
import os, sys
sys.path.insert(0, "."); sys.path.insert(0, "oracle")
import numpy as np
import pgload
pg = pgload.load()
import oracle_py as O
sc = pg.scenes.smoke(96, 96, res=256)
osc = O.OracleScene(pg.capi, sc)
cfg = pg.capi.default_config(integrator=pg.capi.PG_INTEGRATOR_VOLPATH, guiding=1, s_tree_threshold=300.0)
tree = O.OracleSDTree(osc)
for it in range(3):
    st = O.render(osc, cfg, 2 ** it, 2 ** it - 1, record=True, sdtree=tree, nthreads=8)[2]
    tree.splat_pending()
    tree.refit(it, cfg)
rgbw, _, st = O.render(osc, cfg, 16, 7, sdtree=tree, nthreads=8)
print("asan ok: paths", int(st[0]), "segments", int(st[1]), "mean", float(rgbw[..., :3].sum() / rgbw[..., 3].sum()))
PY
