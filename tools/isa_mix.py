"""Static instruction mix of one kernel in an assembly listing (make -C csrc asm).

    python tools/isa_mix.py uu-infogr-raytracer_amd/csrc/obj/rt_kernel.s trace_direct_kernelILi1ELb0ELb0ELi0 [N]
"""
import collections
import sys

L = open(sys.argv[1]).read().split('\n')
key = sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
start = [i for i, l in enumerate(L) if key in l and l.endswith(':') is False and l.startswith('_Z') and ':' in l][0]
end = start + 1
while not L[end].startswith('.Lfunc_end'):
    end += 1
ins = [l.strip().split()[0] for l in L[start:end] if l.startswith('\t') and not l.strip().startswith(('.', ';', '//'))]
c = collections.Counter(ins)
valu = sum(v for k, v in c.items() if k.startswith('v_'))
print(f"{L[start].split(':')[0]}: {len(ins)} instructions, {valu} VALU, {sum(v for k, v in c.items() if k.startswith('s_'))} SALU/branch")
for k, v in c.most_common(top):
    print(f"  {k:28s}{v}")
