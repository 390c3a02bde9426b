// temporary: replay entry points land in replay.cpp
#include "../../include/eao_accel.h"
extern "C" {
int eao_replay_create(eao_assoc*, const char*, int, int, const float*, eao_replay** out) { if (out) *out = nullptr; return EAO_E_STATE; }
int eao_replay_destroy(eao_replay*) { return EAO_OK; }
int eao_replay_frame(eao_replay*, int, const float*, int, const int32_t*, int, const int32_t*, const float*, const float*, const uint8_t*, int32_t*) { return EAO_E_STATE; }
int eao_replay_local_mapping(eao_replay*) { return EAO_E_STATE; }
int eao_replay_num_objects(eao_replay*) { return EAO_E_STATE; }
int eao_replay_object(eao_replay*, int, int32_t*, float*) { return EAO_E_STATE; }
int eao_replay_object_points(eao_replay*, int, int32_t*, int) { return EAO_E_STATE; }
}
