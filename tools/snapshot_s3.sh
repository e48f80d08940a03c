#!/bin/bash
# Snapshot gemm_s3.h at a git revision (default HEAD) as build_variants/gemm_s3_old.h
# with renamed symbols, for tools/gemm_bench.hip -DWITH_OLD (tuning only).
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
mkdir -p "$ROOT/build_variants"
git -C "$ROOT" show "${1:-HEAD}":distributed_ddpg_amd/csrc/gemm_s3.h | sed \
  's/gemm_s3_kernel/gemm_s3old_kernel/g; s/S3_NT/S3O_NT/g; s/struct S3Cfg/struct S3CfgOld/;
   s/S3Cfg</S3CfgOld</g; s/struct StageS3 /struct StageS3Old /; s/StageS3</StageS3Old</g;
   s/split3_pair/split3_pair_old/g; s/widen(/widen_old(/g; s/^typedef __bf16 bf16x2.*//;
   s/^typedef float f32x2v.*//; s/#pragma once//; s/#include "gemm_bf16.h"//;
   s/constexpr int S3_PLANE.*//' > "$ROOT/build_variants/gemm_s3_old.h"
