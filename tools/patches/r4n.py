"""r4n source changes (applied after r4m's snapshot): pipeline skips the CPU
max_len scan of pinned offsets; DG_HOST_NUMA places pinned buffers by the
allocating thread's NUMA policy."""
p = 'dynamicgo_amd/csrc/j2t_pipe.hip'
s = open(p).read()
old = """        uint64_t max_len = 1;
        for (uint64_t j = a; j < a + m; j++) max_len = std::max<uint64_t>(max_len, in_off[j + 1] - in_off[j]);"""
new = """        /* the longest message picks the kernels; unknown (0) when the
         * offsets are pinned: CPU reads of pinned memory run at ~10 GB/s (a
         * 64K batch's offsets cost 50 us), and the kernels route long
         * messages themselves */
        uint64_t max_len = 0;
        if (!zc) {
            max_len = 1;
            for (uint64_t j = a; j < a + m; j++) max_len = std::max<uint64_t>(max_len, in_off[j + 1] - in_off[j]);
        }"""
assert old in s
s = s.replace(old, new)
open(p, 'w').write(s)
p = 'dynamicgo_amd/csrc/host_internal.h'
s = open(p).read()
old = """    HIPCHK(hipHostMalloc((void **)&p, nc, hipHostMallocDefault));
    cap = nc;
    return DG_OK;"""
new = """    /* DG_HOST_NUMA=1: on the allocating thread's NUMA node (its policy)
     * instead of the driver's default placement */
    static const unsigned fl = getenv("DG_HOST_NUMA") ? hipHostMallocNumaUser : hipHostMallocDefault;
    HIPCHK(hipHostMalloc((void **)&p, nc, fl));
    cap = nc;
    return DG_OK;"""
assert old in s
s = s.replace(old, new)
open(p, 'w').write(s)
print("patched")
s = open(p).read()
if "#include <stdlib.h>" not in s:
    s = s.replace("#include <stdint.h>\n", "#include <stdint.h>\n#include <stdlib.h>\n", 1)
    open(p, 'w').write(s)
