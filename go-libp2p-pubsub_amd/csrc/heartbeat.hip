// heartbeat.hip — heartbeat mesh maintenance and message delivery state.
#include <hip/hip_runtime.h>

#include "gsim.h"
#include "gsim_internal.h"

struct Extra {
    int unused = 0;
};

int alloc_extra(gsim_handle* h)
{
    free_extra(h);
    h->x = new Extra();
    return GSIM_OK;
}

void free_extra(gsim_handle* h)
{
    delete h->x;
    h->x = nullptr;
}

bool extra_field_ref(gsim_handle*, int32_t, gsim::FieldRef*) { return false; }
