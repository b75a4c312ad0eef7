#ifndef CLICK_HIPDROPIN_HH
#define CLICK_HIPDROPIN_HH
// The classes hipdropin.cc exports under the reference names (Click's
// generated elements.cc includes the header named after the exporting file).
#include "hipcheck.hh"
#include "hipset.hh"
#include "hipoutput.hh"
#endif
