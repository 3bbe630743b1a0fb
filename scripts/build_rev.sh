#!/usr/bin/env bash
# A/B baseline: variants/<name>/libtpt.so built from git revision REV of the package.
#   scripts/build_rev.sh HEAD base [extra -D flags for the kernel TU]
set -eu
rev=$1; name=$2; shift 2
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d /tmp/tpt_rev.XXXX)
git -C "$root" archive "$rev" toypathtracer-games101-assignment7_amd include | tar -x -C "$tmp"
make -s -C "$tmp/toypathtracer-games101-assignment7_amd" -j8 libtpt.so EXTRA="$*" > /dev/null
mkdir -p "$root/variants/$name"
cp "$tmp/toypathtracer-games101-assignment7_amd/libtpt.so" "$root/variants/$name/libtpt.so"
rm -rf "$tmp"
echo "built $root/variants/$name/libtpt.so from $rev ($*)"
