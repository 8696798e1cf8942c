// rt_kern_core.hip -- the kernels without the extension primitives and materials
// (the build every SURVEY.md 8(d) scene runs).
#define RT_KNS kcore
#define RT_EXT 0
#include "rt_kernels.inc"
