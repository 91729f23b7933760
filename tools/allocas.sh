#!/bin/bash
# Private (scratch) allocas left in one kernel after -O3: bash tools/allocas.sh FILE.hip MANGLED-SUBSTRING
C=$(cd "$(dirname "$0")/.." && pwd)/csrc
/opt/rocm/bin/hipcc -x hip -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -S -emit-llvm "$1" -o /tmp/_allocas.ll \
    -I"$C" -I"$C/codec" -I"$C/runtime" 2>/dev/null || exit 1
python3 - "$2" <<'PY'
import sys
s = open('/tmp/_allocas.ll').read()
i = s.index('define protected amdgpu_kernel void @' + sys.argv[1]) if ('@' + sys.argv[1]) in s else s.index(sys.argv[1])
j = s.index('\n}\n', i)
for l in s[i:j].splitlines():
    if 'alloca' in l:
        print(l.strip()[:160])
PY
