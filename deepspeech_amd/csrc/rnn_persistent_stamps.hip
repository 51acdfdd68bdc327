// Diagnostic build of the persistent recurrence with per-phase s_memtime stamps
// (exports ds2_rnn_fwd_stamps / ds2_rnn_bwd_stamps). Never used on the training path.
#define DS2_RNN_STAMPS 1
#include "rnn_persistent.hip"
