/* TEST INFRASTRUCTURE: shim for libavcodec/decode.h (tests/glue/ffmpeg_decls.h restates what the glue binds) */
#include "ffmpeg_decls.h"
