"""Key of the built library: a hash of the gfx950 code objects inside
libmpgpu.so (its .hip_fatbin section) and of its host code and constants
(.text, .rodata: launch geometry, chunking, stream policy).  profiles/pmc_cfg*.json are keyed by
it, so a comment or documentation change leaves the key alone, a rebuild of
the same sources (the driver rebuilds in its own container) matches, and any
change of the generated kernel code invalidates the recorded counters."""
import hashlib
import os
import struct

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "mplib_amd", "lib", "libmpgpu.so")


def elf_section(path: str, name: str) -> bytes:
    """The bytes of one section of an ELF64 little-endian file."""
    with open(path, "rb") as f:
        data = f.read()
    off, size = elf_section_range(data, name)
    return data[off:off + size]


def elf_section_range(data: bytes, name: str):
    """(file offset, size) of one section of an ELF64 little-endian image."""
    if data[:4] != b"\x7fELF" or data[4] != 2 or data[5] != 1:
        raise ValueError("not an ELF64 little-endian file")
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)

    def sh(i):
        # sh_name, sh_type, sh_flags, sh_addr, sh_offset, sh_size
        return struct.unpack_from("<IIQQQQ", data, shoff + i * shentsize)

    stroff = sh(shstrndx)[4]
    for i in range(shnum):
        nm, _, _, _, off, size = sh(i)
        end = data.index(b"\0", stroff + nm)
        if data[stroff + nm:end].decode() == name:
            return off, size
    raise KeyError(f"no section {name}")


SECTIONS = (".hip_fatbin", ".text", ".rodata")


def build_hash(lib: str = LIB) -> str:
    h = hashlib.sha256()
    for s in SECTIONS:
        h.update(s.encode())
        h.update(elf_section(lib, s))
    return h.hexdigest()[:16]


if __name__ == "__main__":
    import sys
    print(build_hash(*sys.argv[1:]))
