#!/bin/bash
# The shadow pool on one GPU: its parity tests (pytest -k shpool), then same-box A/Bs against persist4 on dragon,
# sportscar and car_boxed (refill thresholds 16 / 8 / 32). Output: gpurun_out/pyt_shp.log, gpurun_out/ab_*.log
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -k shpool -x -q --timeout 300 --timeout-method thread > gpurun_out/pyt_shp.log 2>&1 || { tail -40 gpurun_out/pyt_shp.log; exit 1; }
tail -2 gpurun_out/pyt_shp.log
timeout -k 10 300 python tools/ab_variants.py --frames 16 --rounds 2 persist4 shpool shpool:regroup=8 shpool:regroup=32 > gpurun_out/ab_dragon.log 2>&1 && cat gpurun_out/ab_dragon.log
timeout -k 10 300 python tools/ab_variants.py --scene sportscar --frames 16 --rounds 2 persist4 shpool shpool:regroup=8 shpool:regroup=32 > gpurun_out/ab_sports.log 2>&1 && cat gpurun_out/ab_sports.log
timeout -k 10 300 python tools/ab_variants.py --scene car_boxed --frames 16 --rounds 2 persist4 shpool shpool:regroup=8 shpool:regroup=32 > gpurun_out/ab_car.log 2>&1 && cat gpurun_out/ab_car.log
