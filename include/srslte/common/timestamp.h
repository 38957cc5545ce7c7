/*
 * srslte/common/timestamp.h -- the srsLTE 1.0 timestamp type (full seconds + fractional seconds).
 * srsUE names it in its radio and worker headers (reference ue/hdr/radio/radio.h:32,40-44,
 * ue/hdr/phy/phch_worker.h:53,117) and srslte.h includes it, as srsLTE's does.  The two helpers the
 * sync front end uses are implemented in libsrsue_amd.so (ue_sync.cpp); the rest of srsLTE's
 * timestamp API is only needed by the radio (out of scope).
 */
#ifndef SRSLTE_MI355X_TIMESTAMP_H
#define SRSLTE_MI355X_TIMESTAMP_H
#include <stdint.h>
#include <time.h>
#ifdef __cplusplus
extern "C" {
#endif
typedef struct { time_t full_secs; double frac_secs; } srslte_timestamp_t;
void srslte_timestamp_copy(srslte_timestamp_t *dest, srslte_timestamp_t *src);
int srslte_timestamp_add(srslte_timestamp_t *t, time_t full_secs, double frac_secs);
#ifdef __cplusplus
}
#endif
#endif
