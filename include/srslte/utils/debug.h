/*
 * srslte/utils/debug.h -- the srsLTE 1.0 debug helpers srsUE's PHY worker uses: SRSLTE_DEBUG_ENABLED
 * gates its Error/Warning/Info/Debug macros (reference ue/src/phy/phch_worker.cc:33-36) and
 * get_time_interval times PDCCH / PDSCH decodes under LOG_EXECTIME (:314-315, :351).
 */
#ifndef SRSLTE_MI355X_DEBUG_H
#define SRSLTE_MI355X_DEBUG_H
#include <stdio.h>
#include <sys/time.h>
#ifdef __cplusplus
extern "C" {
#endif
#define SRSLTE_DEBUG_ENABLED 1
#define SRSLTE_VERBOSE_NONE 0
#define SRSLTE_VERBOSE_INFO 1
#define SRSLTE_VERBOSE_DEBUG 2
extern int srslte_verbose;
#define SRSLTE_VERBOSE_ISINFO() (srslte_verbose >= SRSLTE_VERBOSE_INFO)
#define SRSLTE_VERBOSE_ISDEBUG() (srslte_verbose >= SRSLTE_VERBOSE_DEBUG)
/* tdata[0] = tdata[2] - tdata[1] */
void get_time_interval(struct timeval *tdata);
#ifdef __cplusplus
}
#endif
#endif
