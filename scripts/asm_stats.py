"""Per-kernel instruction census of a hipcc -S device assembly file (MFMA, LDS reads, DMA, waits, scratch)."""
import re
import sys

s = open(sys.argv[1]).read()
pat = re.compile(r'\n(_Z\w+):\s*;[^\n]*\n(.*?)\.Lfunc_end', re.S)
for name, body in pat.findall(s):
    if len(sys.argv) > 2 and sys.argv[2] not in name:
        continue
    c = lambda p: len(re.findall(p, body))
    print("%-70s mfma %4d b128 %4d tr %4d flat %3d scratch %3d barrier %3d vmcnt0 %3d vmcntN %3d lgkm %4d dma %3d"
          % (name[-70:], c(r'v_mfma'), c(r'ds_read_b128'), c(r'ds_read_b64_tr_b16'), c(r'\bflat_'),
             c(r'scratch_'), c(r's_barrier'), c(r'vmcnt\(0\)'), c(r'vmcnt\([1-9]'), c(r'lgkmcnt'), c(r'offen lds')))
