/* TEST INFRASTRUCTURE: shim for libavcodec/thread.h (tests/glue/ffmpeg_decls.h restates what the glue binds) */
#include "ffmpeg_decls.h"
