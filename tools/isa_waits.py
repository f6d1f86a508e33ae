"""Print the memory operations and waits of one kernel in a disassembly
(tools/isa.sh output), one per line with its line number, so the vmcnt
waits between a tile's loads and their first use can be read.
usage: isa_waits.py <disassembly> <kernel-name substring> [pattern]"""
import re
import sys

path, want = sys.argv[1], sys.argv[2]
pat = re.compile(sys.argv[3] if len(sys.argv) > 3 else
                 r"(s_waitcnt vmcnt|global_load|global_atomic|global_store|buffer_|scratch_|s_barrier)")
inside = False
for i, line in enumerate(open(path)):
    if line.endswith(">:\n"):
        inside = want in line
        if inside:
            print(line.strip())
        continue
    if inside and pat.search(line):
        print(i, line.split("//")[0].strip())
