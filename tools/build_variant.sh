# Build the working tree's library with extra compile flags into ab/<name>/ (same-box A/B):
#   bash tools/build_variant.sh fwd3 -DATTN_FWD_WPS=3
# (ATTN_FLAGS=... in the environment: flags for attention.hip only)
set -eu
name=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
mkdir -p "$tmp/genomics-lm_amd" "$root/ab/$name"
cp -r "$root/genomics-lm_amd/csrc" "$tmp/genomics-lm_amd/"
cp -r "$root/include" "$tmp/"
make -C "$tmp/genomics-lm_amd/csrc" -j8 OUT="$root/ab/$name/libcodonlm_hip.so" BUILD="$tmp/build" EXTRA_FLAGS="$*" ATTN_FLAGS="${ATTN_FLAGS:-}" > /dev/null
rm -rf "$tmp"
echo "$root/ab/$name/libcodonlm_hip.so"
