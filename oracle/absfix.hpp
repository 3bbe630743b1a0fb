/* Forced-include used ONLY when compiling the reference sources for oracle/_ref
 * (test infrastructure, never shipped).  The reference calls unqualified
 * abs(float|double) in 16 places (e.g. PathTracer.cpp:23, Material.cpp:31);
 * under glibc/libstdc++ those bind to C `int abs(int)` unless std::abs is
 * visible.  MSVC (the author's platform, whose renders are in images/) binds
 * the float overloads; this header reproduces that semantics without editing
 * the reference sources. */
#include <cstdlib>
#include <cmath>
using std::abs;
