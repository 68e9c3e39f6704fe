#!/usr/bin/env bash
# Build a variant of libspi_hip.so for same-process A/B runs (tools/ab_gemm.py,
# tools/gemm_stamps.py).
#   tools/build_variant.sh OUT.so [GIT_REV|WORKTREE] [extra hipcc flags...]
# GIT_REV builds csrc/ and include/ as of that revision; WORKTREE (default)
# builds the current files.  Example:
#   tools/build_variant.sh tools/libspi_ab_old.so HEAD
#   tools/build_variant.sh tools/libspi_stamps.so WORKTREE -DSPI_GEMM_STAMPS
set -euo pipefail
out=$(realpath -m "$1"); rev=${2:-WORKTREE}; shift $(( $# >= 2 ? 2 : 1 ))
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d); trap 'rm -rf "$tmp"' EXIT
mkdir -p "$tmp/pkg/csrc" "$tmp/include"
if [ "$rev" = WORKTREE ]; then
  cp "$root"/starpu-inference-server_amd/csrc/*.{hip,cpp,hpp} "$root"/starpu-inference-server_amd/csrc/Makefile "$tmp/pkg/csrc/"
  cp "$root"/include/*.h "$tmp/include/"
else
  git -C "$root" archive "$rev" starpu-inference-server_amd/csrc include | tar -x -C "$tmp"
  mv "$tmp/starpu-inference-server_amd/csrc/"* "$tmp/pkg/csrc/"
fi
sed -i 's#-I../../include#-I../../include '"$*"'#' "$tmp/pkg/csrc/Makefile"
make -s -C "$tmp/pkg/csrc" -j8 OUT="$out" "$out" >/dev/null
echo "built $out ($rev ${*:-})"
