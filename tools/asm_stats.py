"""Per-kernel statistics from a device-only assembly listing (hipcc --cuda-device-only -S):
VGPR/SGPR/LDS/scratch from the .amdhsa descriptor and counts of interesting instructions.
Usage: python tools/asm_stats.py conv.s [name-substring]"""
import re
import sys


def main():
    s = open(sys.argv[1]).read()
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    for m in re.finditer(r'^(_Z\w+):\s*;', s, re.M):
        name = m.group(1)
        if filt not in name:
            continue
        j = s.find('.Lfunc_end', m.end())
        body = s[m.end():j]
        d = s.find('.amdhsa_kernel ' + name)
        desc = s[d:s.find('.end_amdhsa_kernel', d)]
        g = lambda k: (re.search(k + r'\s+(\d+)', desc) or [None, '?'])[1]
        print(f"{name[-70:]:70s} vgpr {g('.amdhsa_next_free_vgpr')} sgpr {g('.amdhsa_next_free_sgpr')} "
              f"lds {g('.amdhsa_group_segment_fixed_size')} scratch {g('.amdhsa_private_segment_fixed_size')} "
              f"| mfma {body.count('v_mfma')} dma {len(re.findall(r'buffer_load_dwordx4.* lds', body))} "
              f"vmcnt {len(re.findall(r's_waitcnt vmcnt', body))} barrier {body.count('s_barrier')} "
              f"ds_read {len(re.findall(r'ds_read', body))} lines {body.count(chr(10))}")


if __name__ == "__main__":
    main()
