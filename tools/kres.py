"""Print per-kernel resources (LDS, VGPR, SGPR, scratch) of a hipcc --save-temps .s file."""
import re
import sys

s = open(sys.argv[1]).read()
for b in s.split("  - .agpr_count")[1:]:
    def g(k):
        return re.search(k + r":\s+(\d+)", b).group(1)
    name = re.search(r"\.name:\s+(\S+)", b).group(1)
    print(f"{name[:64]:64s} lds={g('group_segment_fixed_size'):>6} vgpr={g('vgpr_count'):>3} "
          f"sgpr={g('sgpr_count'):>3} scratch={g('private_segment_fixed_size')}")
