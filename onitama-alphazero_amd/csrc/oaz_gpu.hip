// oaz_gpu.hip — one translation unit for the rules / search kernels (oaz_kernels.hip), the network
// kernels (oaz_nn.hip) and the one-launch small-batch search (oaz_search_lat.hip), which inlines the
// device bodies of both (tree walk + network in one workgroup).
#include "oaz_kernels.hip"
#include "oaz_nn.hip"
#include "oaz_search_lat.hip"
