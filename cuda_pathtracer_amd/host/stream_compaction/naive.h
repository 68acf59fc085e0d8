// Forwarding header: the reference's include path <stream_compaction/naive.h>, so code written against
// stream_compaction/stream_compaction/naive.h (Naive::scan)
// builds against the mirror with only -I cuda_pathtracer_amd/host (stream_compaction/src/main.cpp:2-5's
// include block unchanged).  Every namespace is declared in ../stream_compaction.h.
#pragma once
#include "../stream_compaction.h"
