// .rten model loader (src/model.rs:265-522): see rtenhip_model_load.
#include "graph.h"

using namespace rtenhip;

extern "C" {

rtenhip_graph* rtenhip_model_load(rtenhip_ctx* ctx, const uint8_t* bytes, size_t len) {
  (void)ctx;
  (void)bytes;
  (void)len;
  set_error(RTENHIP_UNSUPPORTED_VALUE, ".rten loading is not implemented yet");
  return nullptr;
}

}  // extern "C"
