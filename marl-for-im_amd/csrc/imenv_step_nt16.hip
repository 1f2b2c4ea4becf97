// Step kernel instantiations for node capacity 16 (see imenv_step_inst.h).
#define IMENV_NT 16
#include "imenv_step_inst.h"
