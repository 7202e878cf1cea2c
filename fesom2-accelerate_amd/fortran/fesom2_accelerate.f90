! fesom2_accelerate.f90 -- ISO_C_BINDING interface of libfesom2-accelerate.so for FESOM2's Fortran
! host: the entry points of the reference's include/fesom2-accelerate.h:142-236 (same names,
! every argument by reference, device buffers as opaque c_ptr handles) and the additions this
! library makes (c-step, direction-split pass, device residency, downloads, frees).
! Declarations follow include/fesom2-accelerate.h of this repository line by line.
module fesom2_accelerate
  use iso_c_binding
  implicit none
  interface
    ! ---- reference entry points (reference include/fesom2-accelerate.h:146-158)
    subroutine set_mpi_rank(rank, total_ranks) bind(C, name="set_mpi_rank_")
      import :: c_int
      integer(c_int) :: rank, total_ranks
    end subroutine
    subroutine transfer_mesh(handle, host, n, istat) bind(C, name="transfer_mesh_")
      import :: c_ptr, c_int
      type(c_ptr) :: handle
      integer(c_int) :: host(*), n, istat
    end subroutine
    subroutine alloc_var(handle, host, n, create_event, istat) bind(C, name="alloc_var_")
      import :: c_ptr, c_int, c_double, c_bool
      type(c_ptr) :: handle
      real(c_double) :: host(*)
      integer(c_int) :: n, istat
      logical(c_bool) :: create_event
    end subroutine
    subroutine reserve_var(handle, n, create_event, istat) bind(C, name="reserve_var_")
      import :: c_ptr, c_int, c_bool
      type(c_ptr) :: handle
      integer(c_int) :: n, istat
      logical(c_bool) :: create_event
    end subroutine
    subroutine transfer_var(handle, host) bind(C, name="transfer_var_")
      import :: c_ptr, c_double
      type(c_ptr) :: handle
      real(c_double) :: host(*)
    end subroutine
    subroutine transfer_var_async(handle, host, stream, record_event) bind(C, name="transfer_var_async_")
      import :: c_ptr, c_double, c_bool
      type(c_ptr) :: handle, stream
      real(c_double) :: host(*)
      logical(c_bool) :: record_event
    end subroutine
    subroutine fesom2_transfer_back_async(handle, host, stream, istat) bind(C, name="fesom2_transfer_back_async_")
      import :: c_ptr, c_double, c_int
      type(c_ptr) :: handle, stream
      real(c_double) :: host(*)
      integer(c_int) :: istat
    end subroutine
    subroutine make_stream(stream, istat) bind(C, name="make_stream_")
      import :: c_ptr, c_int
      type(c_ptr) :: stream
      integer(c_int) :: istat
    end subroutine
    subroutine await_stream(stream, istat) bind(C, name="await_stream_")
      import :: c_ptr, c_int
      type(c_ptr) :: stream
      integer(c_int) :: istat
    end subroutine
    subroutine fct_ale_pre_comm_acc(alg_state, s, fct_ttf_max, fct_ttf_min, fct_plus, fct_minus, ttf, fct_LO, &
        fct_adf_v, fct_adf_h, UV_rhs, area_inv, myDim_nod2D, eDim_nod2D, myDim_elem2D, myDim_edge2D, nl, &
        nlevels_nod2D, nlevels_elem2D, elem2D_nodes, nod_in_elem2D_num, nod_in_elem2D, nod_in_elem2D_dim, &
        nod2D_edges, elem2D_edges, vlimit, flux_eps, bignumber, dt) bind(C, name="fct_ale_pre_comm_acc_")
      import :: c_ptr, c_int, c_double
      integer(c_int) :: alg_state, myDim_nod2D, eDim_nod2D, myDim_elem2D, myDim_edge2D, nl, nod_in_elem2D_dim, vlimit
      type(c_ptr) :: s, fct_ttf_max, fct_ttf_min, fct_plus, fct_minus, ttf, fct_LO, fct_adf_v, fct_adf_h, UV_rhs, &
                     area_inv, nlevels_nod2D, nlevels_elem2D, elem2D_nodes, nod_in_elem2D_num, nod_in_elem2D, &
                     nod2D_edges, elem2D_edges
      real(c_double) :: flux_eps, bignumber, dt
    end subroutine
    subroutine fct_ale_inter_comm_acc(alg_state, s, fct_plus, fct_minus, fct_adf_v, myDim_nod2D, nl, &
        nlevels_nod2D) bind(C, name="fct_ale_inter_comm_acc_")
      import :: c_ptr, c_int
      integer(c_int) :: alg_state, myDim_nod2D, nl
      type(c_ptr) :: s, fct_plus, fct_minus, fct_adf_v, nlevels_nod2D
    end subroutine
    subroutine fct_ale_post_comm_acc(alg_state, s, fct_plus, fct_minus, fct_adf_h, myDim_edge2D, nl, &
        nlevels_elem2D, nod_in_elem2D_dim, nod2D_edges, elem2D_edges) bind(C, name="fct_ale_post_comm_acc_")
      import :: c_ptr, c_int
      integer(c_int) :: alg_state, myDim_edge2D, nl, nod_in_elem2D_dim
      type(c_ptr) :: s, fct_plus, fct_minus, fct_adf_h, nlevels_elem2D, nod2D_edges, elem2D_edges
    end subroutine
    ! ---- additions: c-step on the GPU (alg_state 9)
    subroutine fct_ale_c_acc(alg_state, s, del_ttf_advvert, del_ttf_advhoriz, ttf, fct_LO, hnode, hnode_new, &
        fct_adf_v, fct_adf_h, area, myDim_nod2D, eDim_nod2D, myDim_edge2D, nl, nlevels_nod2D, nlevels_elem2D, &
        nod2D_edges, elem2D_edges, dt) bind(C, name="fct_ale_c_acc_")
      import :: c_ptr, c_int, c_double
      integer(c_int) :: alg_state, myDim_nod2D, eDim_nod2D, myDim_edge2D, nl
      type(c_ptr) :: s, del_ttf_advvert, del_ttf_advhoriz, ttf, fct_LO, hnode, hnode_new, fct_adf_v, fct_adf_h, &
                     area, nlevels_nod2D, nlevels_elem2D, nod2D_edges, elem2D_edges
      real(c_double) :: dt
    end subroutine
    ! ---- additions: direction-split pass (a1..b2 + b3v + cv, then [exchange] + b3h + ch)
    subroutine fct_ale_pre_comm_v_acc(alg_state, s, ntracers, fct_plus, fct_minus, ttf, fct_LO, fct_adf_v, &
        fct_adf_h, area_inv, area, hnode, hnode_new, del_ttf_advvert, myDim_nod2D, eDim_nod2D, myDim_elem2D, &
        myDim_edge2D, nl, nlevels_nod2D, nlevels_elem2D, elem2D_nodes, nod_in_elem2D_num, nod_in_elem2D, &
        nod_in_elem2D_dim, nod2D_edges, elem2D_edges, vlimit, flux_eps, bignumber, dt) &
        bind(C, name="fct_ale_pre_comm_v_acc_")
      import :: c_ptr, c_int, c_double
      integer(c_int) :: alg_state, ntracers, myDim_nod2D, eDim_nod2D, myDim_elem2D, myDim_edge2D, nl, &
                        nod_in_elem2D_dim, vlimit
      type(c_ptr) :: s, fct_plus, fct_minus, ttf, fct_LO, fct_adf_v, fct_adf_h, area_inv, area, hnode, hnode_new, &
                     del_ttf_advvert, nlevels_nod2D, nlevels_elem2D, elem2D_nodes, nod_in_elem2D_num, &
                     nod_in_elem2D, nod2D_edges, elem2D_edges
      real(c_double) :: flux_eps, bignumber, dt
    end subroutine
    subroutine fct_ale_post_comm_h_acc(alg_state, s, ntracers, comm, halo_plan, fct_plus, fct_minus, fct_adf_h, &
        del_ttf_advhoriz, area, myDim_nod2D, eDim_nod2D, myDim_edge2D, nl, nlevels_nod2D, nlevels_elem2D, &
        nod2D_edges, elem2D_edges, dt) bind(C, name="fct_ale_post_comm_h_acc_")
      import :: c_ptr, c_int, c_double
      integer(c_int) :: alg_state, ntracers, myDim_nod2D, eDim_nod2D, myDim_edge2D, nl
      type(c_ptr) :: s, comm, halo_plan, fct_plus, fct_minus, fct_adf_h, del_ttf_advhoriz, area, nlevels_nod2D, &
                     nlevels_elem2D, nod2D_edges, elem2D_edges
      real(c_double) :: dt
    end subroutine
    ! ---- additions: residency, host copies, release
    subroutine fesom2_set_resident(resident) bind(C, name="fesom2_set_resident_")
      import :: c_int
      integer(c_int) :: resident
    end subroutine
    ! kernel path: 0 fused, 1 stepwise, 2 the reference sequence's fast mode
    subroutine fesom2_set_path(path) bind(C, name="fesom2_set_path_")
      import :: c_int
      integer(c_int) :: path
    end subroutine
    ! fast mode: c-vertical inside fct_ale_pre_comm_acc_ (the c-step's vertical fields bound once)
    subroutine fesom2_bind_c_vertical(istat, fct_adf_v, del_ttf_advvert, hnode, hnode_new, area) &
        bind(C, name="fesom2_bind_c_vertical_")
      import :: c_ptr, c_int
      integer(c_int) :: istat
      type(c_ptr) :: fct_adf_v, del_ttf_advvert, hnode, hnode_new, area
    end subroutine
    subroutine fesom2_download(handle, host, istat) bind(C, name="fesom2_download_")
      import :: c_ptr, c_double, c_int
      type(c_ptr) :: handle
      real(c_double) :: host(*)
      integer(c_int) :: istat
    end subroutine
    subroutine fesom2_upload(handle, host, istat) bind(C, name="fesom2_upload_")
      import :: c_ptr, c_double, c_int
      type(c_ptr) :: handle
      real(c_double) :: host(*)
      integer(c_int) :: istat
    end subroutine
    subroutine fesom2_free(handle) bind(C, name="fesom2_free_")
      import :: c_ptr
      type(c_ptr) :: handle
    end subroutine
    subroutine fesom2_free_stream(stream) bind(C, name="fesom2_free_stream_")
      import :: c_ptr
      type(c_ptr) :: stream
    end subroutine
    ! ---- additions: hipGraph capture / replay of a call sequence (device-resident mode)
    subroutine fesom2_graph_begin(istat, s) bind(C, name="fesom2_graph_begin_")
      import :: c_ptr, c_int
      integer(c_int) :: istat
      type(c_ptr) :: s
    end subroutine
    subroutine fesom2_graph_end(istat, s, graph) bind(C, name="fesom2_graph_end_")
      import :: c_ptr, c_int
      integer(c_int) :: istat
      type(c_ptr) :: s, graph
    end subroutine
    subroutine fesom2_graph_launch(istat, graph, s) bind(C, name="fesom2_graph_launch_")
      import :: c_ptr, c_int
      integer(c_int) :: istat
      type(c_ptr) :: graph, s
    end subroutine
    subroutine fesom2_graph_free(graph) bind(C, name="fesom2_graph_free_")
      import :: c_ptr
      type(c_ptr) :: graph
    end subroutine
  end interface
end module fesom2_accelerate
