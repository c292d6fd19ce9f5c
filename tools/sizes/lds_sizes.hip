// LDS bytes per frame of the scan kernel's configurations (the one-CU-per-frame
// layout): host-side sizeof of Scan2Shared, for DESIGN.md's occupancy
// arithmetic (two frames per CU need <= 80 KB each of the 160 KB).
//   tools/sizes/lds_sizes.sh
#include "../../soundchunks_amd/csrc/gsc_scan.hip"
#include <cstdio>
int main() {
    std::printf("Scan2Shared bytes (LDS per frame; 160 KB = 163840 per CU)\n");
    std::printf("  D=8  K=4096 SL=8      %zu\n", sizeof(Scan2Shared<ScanCfg<8, 12, 8>>));
    std::printf("  D=16 K=4096 SL=8      %zu\n", sizeof(Scan2Shared<ScanCfg<16, 12, 8>>));
    std::printf("  D=32 K=4096 split     %zu\n", sizeof(Scan2Shared<ScanCfg<32, 12, 8, 16>>));
    std::printf("  D=8  K=512  SL=1      %zu\n", sizeof(Scan2Shared<ScanCfg<8, 9, 1>>));
    std::printf("  of which KdTree       %zu (cut value, cell bounds, cut dimension per split node; leaf ids)\n",
                sizeof(KdTree));
    std::printf("  wave records D=8 K=4096  %zu\n", sizeof(WaveRecT<8>) * 8 * 33);
    return 0;
}
