/* TEST INFRASTRUCTURE: shim for libavutil/common.h (tests/glue/ffmpeg_decls.h restates what the glue binds) */
#include "ffmpeg_decls.h"
