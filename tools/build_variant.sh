#!/bin/bash
# Build a variant of libtts_hip.so into variants/lib_<name>.so from the in-tree sources with some
# files replaced:  tools/build_variant.sh <name> <src-file>=<replacement> ...   (CPU, build only)
set -e
name=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
W=$R/your-voice-tts_amd/csrc_var_$name
rm -rf "$W" && cp -r "$R/your-voice-tts_amd/csrc" "$W" && rm -rf "$W/build"
for kv in "$@"; do cp "${kv#*=}" "$W/${kv%%=*}"; done
OUTD=${OUTD:-variants}
mkdir -p "$R/$OUTD"
make -C "$W" -j8 OUT="$R/$OUTD/lib_$name.so" >/dev/null
rm -rf "$W"
echo "$OUTD/lib_$name.so"
