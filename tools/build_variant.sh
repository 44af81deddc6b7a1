#!/bin/bash
# Build another version of the engine library for same-box A/B runs
# (tools/gpu_session.sh ab_* steps):
#
#   tools/build_variant.sh NAME [GITREF]   (default HEAD)
#
# -> primesim_amd/libprimeuncore_NAME.so, built from GITREF's sources in a
# scratch worktree (so it embeds that commit's engine for its compiled
# configuration), with the C4 configuration compiled into
# primesim_amd/jit_cache (jit.cpp keys code objects by source, so the
# variants' code objects sit beside the product library's).  The variant must
# share the product's C ABI (bench.py drives it through primesim_amd/uncore.py).
set -e
NAME=$1; REF=${2:-HEAD}
[ -n "$NAME" ] || { echo "usage: $0 NAME [GITREF]"; exit 2; }
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=$(mktemp -d /tmp/pu_variant_XXXXXX)
git -C "$ROOT" worktree add -f --detach "$WT" "$REF" > /dev/null
trap 'git -C "$ROOT" worktree remove --force "$WT"' EXIT
make -C "$WT/primesim_amd/csrc" -j8 ../libprimeuncore.so > "$WT/build.log" 2>&1 || { tail -20 "$WT/build.log"; exit 1; }
cp "$WT/primesim_amd/libprimeuncore.so" "$ROOT/primesim_amd/libprimeuncore_$NAME.so"
PRIMEUNCORE_JIT_OFFLINE=1 PRIMEUNCORE_LIB="$ROOT/primesim_amd/libprimeuncore_$NAME.so" python3 - "$ROOT" <<'EOF'
import ctypes as C, sys
sys.path.insert(0, sys.argv[1])
import primesim_amd as P
from primesim_amd import config as CF, uncore
rc = uncore.lib().pu_config_jit_warm(C.byref(P.config_from_dict(CF.preset("C4"))))
sys.exit(0 if rc >= 0 else 1)
EOF
echo "built primesim_amd/libprimeuncore_$NAME.so from $(git -C "$ROOT" rev-parse --short "$REF")"
