/*
 * mcs_common.h -- shared status codes / version of the MI355X-native MultiCol-SLAM
 * front-end + BA library (libmcs_amd.so).  No reference interface is replaced here;
 * the reference signals errors by silent early return (e.g.
 * src/mdBRIEFextractorOct.cpp:1252-1253) or cout, the C-ABI uses status codes.
 */
#ifndef MCS_COMMON_H
#define MCS_COMMON_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum mcs_status {
  MCS_OK = 0,
  MCS_ERR_ARG = -1,         /* invalid argument / shape */
  MCS_ERR_CAPACITY = -2,    /* caller buffer too small; required size reported */
  MCS_ERR_HIP = -3,         /* HIP runtime error */
  MCS_ERR_UNSUPPORTED = -4, /* option accepted by the reference but not built yet */
  MCS_ERR_NO_DEVICE = -5    /* no gfx950 device visible */
} mcs_status;

/* Library version string and the last HIP error text (thread-local). */
const char* mcs_version(void);
const char* mcs_last_error(void);
/* Number of visible HIP devices (0 on a GPU-less host; never initialises a context). */
int32_t mcs_device_count(void);

#ifdef __cplusplus
}
#endif
#endif /* MCS_COMMON_H */
