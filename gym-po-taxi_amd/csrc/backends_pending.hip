#include "gp_internal.h"
std::unique_ptr<EnvBackend> make_anttag_backend(const gp_anttag_config*, int64_t, int, int, int* err) { gp_set_error("anttag: not built"); *err = GP_E_UNSUPPORTED; return nullptr; }
