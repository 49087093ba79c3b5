/* tools/variant_stub.c -- linked into A/B variant libraries (tools/build_prev.sh)
 * built from revisions older than an ABI entry point the Python binding binds:
 * weak definitions, so a revision that has the function keeps its own. */
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>

__attribute__((weak)) const char *snappy_amd_build_config(void) { return "variant (revision without a build config)"; }
