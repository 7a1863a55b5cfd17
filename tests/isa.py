"""gfx950 ISA of the built libdlagg.so: pull the code object out of the .hip_fatbin clang
offload bundle and disassemble it with ROCm's llvm-objdump (test helper, CPU only)."""
import os
import re
import struct
import subprocess
import tempfile
from typing import Dict, List

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def gfx950_code_object(so_path: str) -> bytes:
    out = subprocess.run([READELF, "-S", "--wide", so_path], capture_output=True, text=True, check=True).stdout
    m = re.search(r"\.hip_fatbin\s+PROGBITS\s+[0-9a-f]+\s+([0-9a-f]+)\s+([0-9a-f]+)", out)
    if not m:
        raise RuntimeError("no .hip_fatbin section in %s" % so_path)
    off, size = int(m.group(1), 16), int(m.group(2), 16)
    with open(so_path, "rb") as f:
        f.seek(off)
        sec = f.read(size)
    if not sec.startswith(_MAGIC):
        raise RuntimeError("unexpected fat-binary format (compressed bundle?)")
    n = struct.unpack_from("<Q", sec, len(_MAGIC))[0]
    pos = len(_MAGIC) + 8
    for _ in range(n):
        o, sz, tl = struct.unpack_from("<QQQ", sec, pos)
        pos += 24
        triple = sec[pos:pos + tl].decode()
        pos += tl
        if triple.endswith("gfx950"):
            return sec[o:o + sz]
    raise RuntimeError("no gfx950 code object in %s" % so_path)


def disassemble(so_path: str) -> Dict[str, List[str]]:
    """{mangled function name: [instruction lines]} of the gfx950 code object."""
    with tempfile.NamedTemporaryFile(suffix=".co") as tmp:
        tmp.write(gfx950_code_object(so_path))
        tmp.flush()
        text = subprocess.run([OBJDUMP, "-d", tmp.name], capture_output=True, text=True, check=True).stdout
    funcs: Dict[str, List[str]] = {}
    cur = None
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            cur = funcs.setdefault(m.group(1), [])
        elif cur is not None and line.strip():
            cur.append(line.split("//")[0].strip())
    return funcs


def available() -> bool:
    return os.path.exists(OBJDUMP) and os.path.exists(READELF)
