// Instantiations of the SGNS kernels for VEC = 8 (d in (256, 512]).
#include "come_sgns_impl.h"

namespace come {

const KernelSet &kernels_vec8() {
    static KernelSet ks = [] {
        KernelSet k{};
        k.o2_direct[0][0] = (void *)&k_sgns_o2<8, false, 5>;
        k.o1[0][0] = (void *)&k_sgns_o1<8, false, 5>;
        k.o1_runs[0][0] = (void *)&k_sgns_o1_runs<8, false, 5>;
        k.o2_ring[0][0] = (void *)&k_sgns_o2_ring<8, false, 5>;
        k.o2_stream[0][0] = (void *)&k_sgns_o2_stream<8, false, 5>;
        k.o2_direct[0][1] = (void *)&k_sgns_o2<8, false, 10>;
        k.o1[0][1] = (void *)&k_sgns_o1<8, false, 10>;
        k.o1_runs[0][1] = (void *)&k_sgns_o1_runs<8, false, 10>;
        k.o2_ring[0][1] = (void *)&k_sgns_o2_ring<8, false, 10>;
        k.o2_stream[0][1] = (void *)&k_sgns_o2_stream<8, false, 10>;
        k.o2_direct[0][2] = (void *)&k_sgns_o2<8, false, 20>;
        k.o1[0][2] = (void *)&k_sgns_o1<8, false, 20>;
        k.o1_runs[0][2] = (void *)&k_sgns_o1_runs<8, false, 20>;
        k.o2_ring[0][2] = (void *)&k_sgns_o2_ring<8, false, 20>;
        k.o2_stream[0][2] = (void *)&k_sgns_o2_stream<8, false, 20>;
        k.o2_direct[1][0] = (void *)&k_sgns_o2<8, true, 5>;
        k.o1[1][0] = (void *)&k_sgns_o1<8, true, 5>;
        k.o1_runs[1][0] = (void *)&k_sgns_o1_runs<8, true, 5>;
        k.o2_ring[1][0] = (void *)&k_sgns_o2_ring<8, true, 5>;
        k.o2_stream[1][0] = (void *)&k_sgns_o2_stream<8, true, 5>;
        k.o2_direct[1][1] = (void *)&k_sgns_o2<8, true, 10>;
        k.o1[1][1] = (void *)&k_sgns_o1<8, true, 10>;
        k.o1_runs[1][1] = (void *)&k_sgns_o1_runs<8, true, 10>;
        k.o2_ring[1][1] = (void *)&k_sgns_o2_ring<8, true, 10>;
        k.o2_stream[1][1] = (void *)&k_sgns_o2_stream<8, true, 10>;
        k.o2_direct[1][2] = (void *)&k_sgns_o2<8, true, 20>;
        k.o1[1][2] = (void *)&k_sgns_o1<8, true, 20>;
        k.o1_runs[1][2] = (void *)&k_sgns_o1_runs<8, true, 20>;
        k.o2_ring[1][2] = (void *)&k_sgns_o2_ring<8, true, 20>;
        k.o2_stream[1][2] = (void *)&k_sgns_o2_stream<8, true, 20>;
        return k;
    }();
    return ks;
}

hipError_t upload_exp_table_vec8(const float *host1000) {
    return hipMemcpyToSymbol(HIP_SYMBOL(c_exp_table), host1000, sizeof(float) * kExpTableSize);
}

}  // namespace come
