// Variant build (tools/build_variant.sh): single-frame fetches wait on the stream instead of
// polling the split launch's done word (the stream wait alone).
//   VARIANT=tools/variants/no_done_word.h tools/build_variant.sh nodone
#define CG_HOOK_POLL_DONE_WORD 0
