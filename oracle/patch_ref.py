#!/usr/bin/env python3
"""TEST INFRASTRUCTURE: build the reference simulator as a benchmark binary.

Reads /root/reference/assignment.c where it lies, applies the minimal patch of
SURVEY.md §8(d) / BASELINE.md to a copy in a temporary directory (never inside
this repository), and compiles it with `gcc -O2 -fopenmp` into
oracle/_ref/cache_simulator_bench (git-ignored; it travels to the GPU box like
the other built files). Only bench.py's cpu_baseline leg runs it.

The patch (each edit is anchored on text that must occur exactly once):
  1. NUM_PROCS, CACHE_SIZE, MAX_INSTR_NUM become -D overridable (ref :6-10);
  2. the queue count is atomic on both sides -- dequeue `count--` (ref :177) and
     enqueue `count++` (ref :757) -- and the consumer's `count > 0` test is an
     atomic load (ref :169); without this, 4096-instruction runs hang;
  3. sendMessage drops a message to a receiver >= NUM_PROCS (ref :751; the
     0xFF-line eviction of ref :772,786 would index messageBuffers[15]);
  4. termination: a global in-flight counter (incremented on every successful
     enqueue, decremented after a message's handler finishes, ref :619) and a
     count of threads whose instructions are all done; a thread that has printed
     its final state (ref :632-646) exits once every thread is done and nothing
     is in flight. The unpatched program never exits (ref :165).
  5. (round 6) the first send of each message type that patch 3 drops, and the first of each type
     that a full queue drops (ref :758-762), is noted on stderr as
     `bench: dropped <type> to node <receiver>` / `bench: queue full at node <receiver>, dropped
     <type>`, so bench.py can say why an instance it killed had stalled (a WRITEBACK_INT /
     WRITEBACK_INV sent to node 32 is the reference's __builtin_ctz(0), ref :209,451: its requester
     then waits forever). Only the drop paths print; the handlers are untouched.
  6. (round 6) SIGUSR1 prints one snapshot line on stderr -- `bench: snapshot done <threads done>
     inflight <messages in flight> q<n>:<head>,<tail>,<count> ...` for every queue -- from an
     async-signal-safe handler reading the globals (ref :102 and patch 4's counters). bench.py
     sends it twice, a second apart, to an instance that outlives the batch: unchanged snapshots
     mean no message moved (stalled, killed); changed ones mean a slow instance, which is waited
     for. Nothing on the simulation path changes.
Everything else -- the handlers, locks, spinning, state dumps -- is the reference.
"""
import pathlib
import subprocess
import sys
import tempfile

EDITS = [
    ("#define NUM_PROCS 4\n", "#ifndef NUM_PROCS\n#define NUM_PROCS 4\n#endif\n"),
    ("#define CACHE_SIZE 4\n", "#ifndef CACHE_SIZE\n#define CACHE_SIZE 4\n#endif\n"),
    ("#define MAX_INSTR_NUM 32\n", "#ifndef MAX_INSTR_NUM\n#define MAX_INSTR_NUM 32\n#endif\n"),
    ("omp_lock_t msgBufferLocks[ NUM_PROCS ];\n",
     "omp_lock_t msgBufferLocks[ NUM_PROCS ];\n"
     "static long bench_inflight = 0;  /* patch 4 */\n"
     "static int bench_done = 0;\n"
     "static unsigned bench_noted = 0;  /* patch 5 */\n"
     "static void bench_note_drop( int receiver, int type, int full ) {\n"
     "    unsigned bit = 1u << ( ( type & 15 ) + ( full ? 16 : 0 ) );\n"
     "    if ( __atomic_fetch_or( &bench_noted, bit, __ATOMIC_SEQ_CST ) & bit ) return;\n"
     "    if ( full ) fprintf( stderr, \"bench: queue full at node %d, dropped %d\\n\", receiver, type );\n"
     "    else fprintf( stderr, \"bench: dropped %d to node %d\\n\", type, receiver );\n"
     "}\n"
     "#include <signal.h>\n"
     "#include <unistd.h>\n"
     "static void bench_put( char **p, const char *s, long v ) {  /* patch 6 */\n"
     "    char t[24]; int n = 0;\n"
     "    while ( *s ) *( *p )++ = *s++;\n"
     "    if ( v < 0 ) { *( *p )++ = '-'; v = -v; }\n"
     "    do { t[ n++ ] = (char)( '0' + v % 10 ); v /= 10; } while ( v );\n"
     "    while ( n ) *( *p )++ = t[ --n ];\n"
     "}\n"
     "static void bench_snapshot( int sig ) {\n"
     "    char buf[ 64 + 48 * NUM_PROCS ], *p = buf;\n"
     "    (void)sig;\n"
     "    bench_put( &p, \"bench: snapshot done \", __atomic_load_n( &bench_done, __ATOMIC_SEQ_CST ) );\n"
     "    bench_put( &p, \" inflight \", __atomic_load_n( &bench_inflight, __ATOMIC_SEQ_CST ) );\n"
     "    for ( int i = 0; i < NUM_PROCS; i++ ) {\n"
     "        bench_put( &p, \" q\", i );\n"
     "        bench_put( &p, \":\", messageBuffers[ i ].head );\n"
     "        bench_put( &p, \",\", messageBuffers[ i ].tail );\n"
     "        bench_put( &p, \",\", __atomic_load_n( &messageBuffers[ i ].count, __ATOMIC_SEQ_CST ) );\n"
     "    }\n"
     "    *p++ = '\\n';\n"
     "    ssize_t w = write( 2, buf, (size_t)( p - buf ) );\n"
     "    (void)w;\n"
     "}\n"),
    ("                messageBuffers[ threadId ].count > 0 &&",
     "                __atomic_load_n( &messageBuffers[ threadId ].count, __ATOMIC_SEQ_CST ) > 0 &&"),
    ("                messageBuffers[ threadId ].count--;\n",
     "                __atomic_fetch_sub( &messageBuffers[ threadId ].count, 1, __ATOMIC_SEQ_CST );\n"),
    ("                        break;\n                }\n            }\n            \n"
     "            // Check if we are waiting for a reply message",
     "                        break;\n                }\n"
     "                __atomic_fetch_sub( &bench_inflight, 1, __ATOMIC_SEQ_CST );\n"
     "            }\n            \n            // Check if we are waiting for a reply message"),
    ("        byte waitingForReply = 0;",
     "        int benchFinished = 0;\n        byte waitingForReply = 0;"),
    ("                    printProcessorState( threadId, node );\n                    printProcState--;\n"
     "                }\n",
     "                    printProcessorState( threadId, node );\n                    printProcState--;\n"
     "                }\n"
     "                if ( !benchFinished ) {\n"
     "                    benchFinished = 1;\n"
     "                    __atomic_fetch_add( &bench_done, 1, __ATOMIC_SEQ_CST );\n"
     "                }\n"
     "                if ( __atomic_load_n( &bench_done, __ATOMIC_SEQ_CST ) == NUM_PROCS &&\n"
     "                     __atomic_load_n( &bench_inflight, __ATOMIC_SEQ_CST ) == 0 )\n"
     "                    break;\n"),
    ("    omp_set_lock( &msgBufferLocks[ receiver ] );\n",
     "    if ( receiver < 0 || receiver >= NUM_PROCS ) {  /* patch 3 */\n"
     "        bench_note_drop( receiver, msg.type, 0 );\n"
     "        return;\n"
     "    }\n"
     "    omp_set_lock( &msgBufferLocks[ receiver ] );\n"),
    ("      buf->count++;\n",
     "      __atomic_fetch_add( &bench_inflight, 1, __ATOMIC_SEQ_CST );\n"
     "      __atomic_fetch_add( &buf->count, 1, __ATOMIC_SEQ_CST );\n"),
    ("    omp_set_num_threads(NUM_PROCS);\n",
     "    omp_set_num_threads(NUM_PROCS);\n    signal( SIGUSR1, bench_snapshot );  /* patch 6 */\n"),
    ("    } else {\n#ifdef DEBUG\n        fprintf(stderr, \"Error: Message buffer overflow",
     "    } else {\n        bench_note_drop( receiver, msg.type, 1 );  /* patch 5 */\n"
     "#ifdef DEBUG\n        fprintf(stderr, \"Error: Message buffer overflow"),
]


# (output name, -D flags). The bench binaries: 8 nodes, 4096 instructions, one per CACHE_SIZE of
# BASELINE configs[4] (bench.py's cpu_baseline; CACHE_SIZE 4 keeps the round-2 name). The pin
# binaries: the reference's own 4 nodes / 32 instructions with its DEBUG_MSG trace of every handled
# message (ref :179-182), for tests/test_reference_cross_node.py (the oracle's cross-node handlers
# checked against the reference itself).
TARGETS = [("cache_simulator_bench", ["-DNUM_PROCS=8", "-DMAX_INSTR_NUM=4096", "-DCACHE_SIZE=4"])]
TARGETS += [(f"cache_simulator_bench_cs{cs}", ["-DNUM_PROCS=8", "-DMAX_INSTR_NUM=4096", f"-DCACHE_SIZE={cs}"])
            for cs in (1, 2, 8, 16)]
TARGETS += [(f"cache_simulator_pin_cs{cs}", ["-DNUM_PROCS=4", "-DMAX_INSTR_NUM=32", f"-DCACHE_SIZE={cs}",
                                              "-DDEBUG_MSG", "-DDEBUG_INSTR"]) for cs in (1, 4)]
# the same at the headline's 8 nodes (round 3): cross-node traffic among 8 homes. Round 4: DEBUG_INSTR
# too, so each thread's whole event log (pops and issues, ref :179-182, :649-652) is printed and the
# oracle replays it (tests/ref_pin.py guided pin)
TARGETS += [(f"cache_simulator_pin8_cs{cs}", ["-DNUM_PROCS=8", "-DMAX_INSTR_NUM=32", f"-DCACHE_SIZE={cs}",
                                               "-DDEBUG_MSG", "-DDEBUG_INSTR"]) for cs in (1, 4)]


def main():
    ref = pathlib.Path(sys.argv[1] if len(sys.argv) > 1 else "/root/reference") / "assignment.c"
    outdir = pathlib.Path(__file__).resolve().parent / "_ref"
    if not ref.exists():
        print(f"reference not present at {ref}; skipping", file=sys.stderr)
        return 0
    src = ref.read_text()
    for old, new in EDITS:
        n = src.count(old)
        if n != 1:
            raise SystemExit(f"patch anchor found {n} times: {old[:60]!r}")
        src = src.replace(old, new)
    outdir.mkdir(parents=True, exist_ok=True)
    with tempfile.TemporaryDirectory() as td:
        c = pathlib.Path(td) / "assignment_bench.c"
        c.write_text(src)
        for name, defs in TARGETS:
            out = outdir / name
            subprocess.run(["gcc", "-O2", "-fopenmp", "-w"] + defs + ["-o", str(out), str(c)], check=True)
            print(f"built {out}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
