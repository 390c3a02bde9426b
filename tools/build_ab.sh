#!/bin/bash
# Build the engine library of a git revision into eao-slam_amd/lib/ab/<name>/libeao_accel.so (for
# same-box A/B runs with EAO_ACCEL_LIB; development aid). usage: tools/build_ab.sh REV NAME
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
REV=$1; NAME=$2
TMP=$(mktemp -d)
git -C "$ROOT" archive "$REV" eao-slam_amd/csrc eao-slam_amd/Makefile eao-slam_amd/gen_co.py include | tar -x -C "$TMP"
make -s -j8 -C "$TMP/eao-slam_amd" OUT=lib
mkdir -p "$ROOT/eao-slam_amd/lib/ab/$NAME"
cp "$TMP/eao-slam_amd/lib/libeao_accel.so" "$ROOT/eao-slam_amd/lib/ab/$NAME/"
rm -rf "$TMP"
echo "built $ROOT/eao-slam_amd/lib/ab/$NAME/libeao_accel.so ($REV)"
