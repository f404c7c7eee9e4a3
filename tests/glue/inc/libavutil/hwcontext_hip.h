/* TEST INFRASTRUCTURE: libavutil/hwcontext_hip.h is the repository's integration/hwcontext_hip.h */
#include "../../../../integration/hwcontext_hip.h"
