/* Embeds the gfx950 code object built from p1hip_kernels.hip (Makefile:
   build/p1hip_kernels.hsaco) into libp1hip.so; p1hip.hip loads it with
   hipModuleLoadData on every device it initialises. */
    .section .rodata
    .balign 4096
    .globl p1hip_kernels_co
    .type p1hip_kernels_co, @object
p1hip_kernels_co:
    .incbin P1HIP_KERNELS_CO
    .globl p1hip_kernels_co_end
p1hip_kernels_co_end:
    .section .note.GNU-stack,"",@progbits
