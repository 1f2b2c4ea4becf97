// Step kernel instantiations for node capacity 6 (see imenv_step_inst.h).
#define IMENV_NT 6
#include "imenv_step_inst.h"
