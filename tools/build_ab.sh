#!/bin/bash
# Build librsg.so from another git revision of rsync_amd/csrc + include into
# rsync_amd/ab/librsg_<name>.so, for same-box A/B runs (RSG_LIB_PATH).
#   tools/build_ab.sh <rev> <name>
set -e
rev=$1; name=$2
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
mkdir -p "$tmp/rsync_amd/csrc" "$tmp/include" "$root/rsync_amd/ab"
for f in $(git -C "$root" ls-tree --name-only "$rev" rsync_amd/csrc/ include/); do
    git -C "$root" show "$rev:$f" > "$tmp/$f"
done
make -s -C "$tmp/rsync_amd/csrc" -j8 OUT="$root/rsync_amd/ab/librsg_$name.so" OBJDIR="$tmp/obj"
rm -rf "$tmp"
echo "built rsync_amd/ab/librsg_$name.so from $rev"
