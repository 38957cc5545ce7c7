/* TEST STUB (compile check only): the UHD glue type srsUE's radio_uhd.h names
 * (reference ue/hdr/radio/radio_uhd.h:29,85).  Not part of the DL drop-in. */
#pragma once
typedef enum { CUHD_MSG_OK, CUHD_MSG_UNDERFLOW, CUHD_MSG_OVERFLOW, CUHD_MSG_LATE } cuhd_msg_t;
typedef void (*cuhd_msg_handler_t)(const char *);
