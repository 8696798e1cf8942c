// rt_kern_ext.hip -- the kernels with cubes, quads, the quad light, TextureMaterial and
// non-Light light materials (Primitive.h:195-247, TextureMaterial.h).
#define RT_KNS kext
#define RT_EXT 1
#include "rt_kernels.inc"
