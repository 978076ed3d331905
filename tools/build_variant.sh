# Build the working tree's library with extra compile flags into ${VAR_DIR:-ab}/<name>/ (var/ travels to the GPU box, ab/ does not) (same-box A/B):
#   bash tools/build_variant.sh fwd3 -DATTN_FWD_WPS=3
set -eu
if [ -n "${ATTN_FLAGS:-}" ]; then echo "ATTN_FLAGS is gone: pass the flags as arguments (EXTRA_FLAGS)" >&2; exit 2; fi
name=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
out=${VAR_DIR:-ab}
tmp=$(mktemp -d)
mkdir -p "$tmp/genomics-lm_amd" "$root/$out/$name"
cp -r "$root/genomics-lm_amd/csrc" "$tmp/genomics-lm_amd/"
cp -r "$root/include" "$tmp/"
make -C "$tmp/genomics-lm_amd/csrc" -j8 OUT="$root/$out/$name/libcodonlm_hip.so" BUILD="$tmp/build" EXTRA_FLAGS="$*" > /dev/null
rm -rf "$tmp"
echo "$root/$out/$name/libcodonlm_hip.so"
