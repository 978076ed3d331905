# Build the library from a git revision into ab/<name>/libcodonlm_hip.so (for same-box A/B):
#   bash tools/build_base.sh HEAD~1 base
set -eu
rev=${1:-HEAD}; name=${2:-base}
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
git -C "$root" archive "$rev" genomics-lm_amd/csrc include | tar -x -C "$tmp"
mkdir -p "$root/ab/$name"
make -C "$tmp/genomics-lm_amd/csrc" -j8 OUT="$root/ab/$name/libcodonlm_hip.so" BUILD="$tmp/build" > /dev/null
rm -rf "$tmp"
echo "$root/ab/$name/libcodonlm_hip.so"
