/* fast_co.S -- embeds the fast_search code object (fast_search.hip after the
   issue-priority pass, built by the Makefile into build/fast_search.hsaco) in
   libminehip.so.  search_kernels.hip loads it per device (hipModuleLoadData). */
    .section .rodata
    .p2align 12
    .globl mh_fast_co_begin
    .type mh_fast_co_begin, @object
mh_fast_co_begin:
    .incbin "fast_search.hsaco"
    .globl mh_fast_co_end
mh_fast_co_end:
    .size mh_fast_co_begin, mh_fast_co_end - mh_fast_co_begin
    .section .note.GNU-stack,"",@progbits
