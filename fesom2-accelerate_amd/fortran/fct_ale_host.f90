! fct_ale_host.f90 -- a Fortran host that drives libfesom2-accelerate.so the way FESOM2's fct_ale
! does (SURVEY.md 3.1; reference src/fesom2-accelerate.cu:114-379): mesh arrays uploaded once with
! transfer_mesh_, every field bound with alloc_var_ to its Fortran array, scratch with reserve_var_,
! then the phase entries on one stream.  It is the drop-in check in the host language the reference
! serves: built with amdflang, run by tests/test_gpu_fortran.py on a mesh written by Python, its
! outputs compared cell for cell with the oracle.
!
!   fct_ale_host IN OUT
!
! IN  (stream access, little endian): for each array an int64 element count, then the elements:
!     header int32(8) = [myDim_nod2D, eDim_nod2D, myDim_elem2D, myDim_edge2D, nl, nod_in_elem2D_dim,
!     vlimit, mode]; int32 nlevels_nod2D, nlevels_elem2D, elem2D_nodes, nod_in_elem2D_num,
!     nod_in_elem2D, edges, edge_tri; real64 ttf, fct_LO, fct_adf_v, fct_adf_h, area, area_inv, hnode,
!     hnode_new, del_ttf_advvert, del_ttf_advhoriz, [dt, flux_eps, bignumber]
! mode 0: the reference sequence with the reference's transfer semantics (pre_comm -> inter_comm ->
!         post_comm -> c; results land in the bound host arrays)
! mode 1: device resident, direction-split pass (pre_comm_v -> post_comm_h), results downloaded
! mode 2: as 1, the pass captured into a hipGraph (fesom2_graph_*) after one eager pass, replayed
! mode 3: mode 0's unmodified sequence and transfer semantics in the fast mode: fesom2_set_path_(2)
!         and fesom2_bind_c_vertical_ once before the step (b3v, cv and the block-internal edges
!         inside pre_comm, c-horizontal alone in the c-step)
! mode 4: device resident with host-side producer fields (bench.py --transfers producer): the
!         producer's ttf, fct_LO, fct_adf_v, fct_adf_h and the host's del_ttf go up with
!         transfer_var_async_, the direction-split pass runs, and del_ttf_advvert/advhoriz come back
!         with fesom2_transfer_back_async_ (the other outputs are downloaded only for the check)
! Modes 1, 2 and 4 take several tracers at once (FESOM2's tracer loop as one batched call, BASELINE
! config 3): ttf, fct_LO, fct_adf_v, fct_adf_h, del_ttf_advvert and del_ttf_advhoriz then hold
! ntracers Fortran arrays one after another, (nl-1, nod, ntracers) etc.; ntracers = size(ttf) /
! ((myDim+eDim)*(nl-1)).  The mesh fields (area, area_inv, hnode, hnode_new) are shared.
! OUT: int32(4) alg_states, then fct_plus, fct_minus, fct_adf_v, fct_adf_h, del_ttf_advvert,
!      del_ttf_advhoriz in the IN format.
program fct_ale_host
  use iso_c_binding
  use fesom2_accelerate
  implicit none
  integer(c_int) :: hdr(8), N, H, T, E, nl, dim, vlimit, mode, NT, L, istat, st(4), zero, one, two, ntr
  integer(c_int), allocatable, target :: nlev_nod(:), nlev_elem(:), elem_nodes(:), nie_num(:), nie(:), &
                                         edges(:), edge_tri(:)
  real(c_double), allocatable, target :: ttf(:), lo(:), adf_v(:), adf_h(:), area(:), area_inv(:), hnode(:), &
                                         hnode_new(:), del_v(:), del_h(:), plus(:), minus(:), sc(:)
  type(c_ptr) :: s, h_nlev_nod, h_nlev_elem, h_elem_nodes, h_nie_num, h_nie, h_edges, h_edge_tri
  type(c_ptr) :: h_ttf, h_lo, h_adf_v, h_adf_h, h_area, h_area_inv, h_hnode, h_hnode_new, h_del_v, h_del_h, &
                 h_plus, h_minus, h_tmax, h_tmin, h_uv, nullh, graph
  character(len=1024) :: fin, fout
  integer :: u
  logical(c_bool) :: yes, no

  call get_command_argument(1, fin)
  call get_command_argument(2, fout)
  open(newunit=u, file=trim(fin), access='stream', form='unformatted', status='old')
  call read_i(u, hdr)
  N = hdr(1); H = hdr(2); T = hdr(3); E = hdr(4); nl = hdr(5); dim = hdr(6); vlimit = hdr(7); mode = hdr(8)
  NT = N + H; L = nl - 1
  call read_ia(u, nlev_nod); call read_ia(u, nlev_elem); call read_ia(u, elem_nodes)
  call read_ia(u, nie_num); call read_ia(u, nie); call read_ia(u, edges); call read_ia(u, edge_tri)
  call read_ra(u, ttf); call read_ra(u, lo); call read_ra(u, adf_v); call read_ra(u, adf_h)
  call read_ra(u, area); call read_ra(u, area_inv); call read_ra(u, hnode); call read_ra(u, hnode_new)
  call read_ra(u, del_v); call read_ra(u, del_h); call read_ra(u, sc)
  close(u)
  ntr = 1
  if (NT * L > 0) ntr = int(size(ttf) / (NT * L), c_int)
  if (ntr < 1 .or. size(ttf) /= ntr * NT * L .or. ((mode == 0 .or. mode == 3) .and. ntr /= 1)) then
    print *, 'fct_ale_host: ttf holds ', size(ttf), ' values: not a whole number of tracers for mode ', mode
    error stop 4
  end if
  allocate(plus(NT * L * ntr), minus(NT * L * ntr))
  plus = 0; minus = 0
  yes = .true.; no = .false.; zero = 0; one = 1; two = 2; st = -1
  nullh = c_null_ptr

  call set_mpi_rank(zero, one)
  call make_stream(s, istat)
  call check(istat, "make_stream")
  if (mode == 1 .or. mode == 2 .or. mode == 4) call fesom2_set_resident(one)
  ! mesh: once per run (reference .cu:114-127)
  call upload_mesh(h_nlev_nod, nlev_nod); call upload_mesh(h_nlev_elem, nlev_elem)
  call upload_mesh(h_elem_nodes, elem_nodes); call upload_mesh(h_nie_num, nie_num)
  call upload_mesh(h_nie, nie); call upload_mesh(h_edges, edges); call upload_mesh(h_edge_tri, edge_tri)
  ! fields bound to their host arrays (reference .cu:129-141); events on ttf, adf_v, adf_h
  call bind(h_ttf, ttf, yes); call bind(h_lo, lo, no); call bind(h_adf_v, adf_v, yes)
  call bind(h_adf_h, adf_h, yes); call bind(h_area, area, no); call bind(h_area_inv, area_inv, no)
  call bind(h_hnode, hnode, no); call bind(h_hnode_new, hnode_new, no); call bind(h_del_v, del_v, no)
  call bind(h_del_h, del_h, no); call bind(h_plus, plus, no); call bind(h_minus, minus, no)
  call reserve_var(h_tmax, NT * L, no, istat); call check(istat, "reserve_var")
  call reserve_var(h_tmin, NT * L, no, istat); call check(istat, "reserve_var")
  call reserve_var(h_uv, 2 * L * T, no, istat); call check(istat, "reserve_var")
  if (mode == 4) then
    ! bind (alloc_var_) already copied every field up with the same contents: overwrite the device
    ! copies of the fields the step uploads with a sentinel, so a missing or misordered in-step
    ! upload shows in the results (ADVICE r5)
    call poison(h_ttf, size(ttf)); call poison(h_adf_v, size(adf_v)); call poison(h_adf_h, size(adf_h))
    call poison(h_lo, size(lo)); call poison(h_del_v, size(del_v)); call poison(h_del_h, size(del_h))
  end if
  ! per step: the producer's uploads (fct_ale_muscl_LH, reference .cu:269-270)
  call transfer_var_async(h_ttf, ttf, s, yes)
  call transfer_var_async(h_adf_v, adf_v, s, yes)
  call transfer_var_async(h_adf_h, adf_h, s, yes)

  if (mode == 3) then
    call fesom2_set_path(two)
    call fesom2_bind_c_vertical(istat, h_adf_v, h_del_v, h_hnode, h_hnode_new, h_area)
    call check(istat, "fesom2_bind_c_vertical")
  end if
  if (mode == 0 .or. mode == 3) then
    call fct_ale_pre_comm_acc(st(1), s, h_tmax, h_tmin, h_plus, h_minus, h_ttf, h_lo, h_adf_v, h_adf_h, h_uv, &
        h_area_inv, N, H, T, E, nl, h_nlev_nod, h_nlev_elem, h_elem_nodes, h_nie_num, h_nie, dim, h_edges, &
        h_edge_tri, vlimit, sc(2), sc(3), sc(1))
    call await_stream(s, istat)
    ! exchange_nod(fct_plus, fct_minus) would run here (one rank: nothing to exchange)
    call fct_ale_inter_comm_acc(st(2), s, h_plus, h_minus, h_adf_v, N, nl, h_nlev_nod)
    call fct_ale_post_comm_acc(st(3), s, h_plus, h_minus, h_adf_h, E, nl, h_nlev_elem, dim, h_edges, h_edge_tri)
    call fct_ale_c_acc(st(4), s, h_del_v, h_del_h, h_ttf, h_lo, h_hnode, h_hnode_new, h_adf_v, h_adf_h, h_area, &
        N, H, E, nl, h_nlev_nod, h_nlev_elem, h_edges, h_edge_tri, sc(1))
    call await_stream(s, istat)
    call check(istat, "await_stream")
  else
    if (mode == 2) then
      ! one eager pass builds the mesh plans, the pristine inputs go back up, and the pass is
      ! captured into a hipGraph that the replay below runs instead of the entry calls
      call split_pass()
      call await_stream(s, istat)
      call transfer_var(h_adf_v, adf_v); call transfer_var(h_adf_h, adf_h)
      call transfer_var(h_del_v, del_v); call transfer_var(h_del_h, del_h)
      call fesom2_graph_begin(istat, s); call check(istat, "fesom2_graph_begin")
      call split_pass()
      call fesom2_graph_end(istat, s, graph); call check(istat, "fesom2_graph_end")
      call fesom2_graph_launch(istat, graph, s); call check(istat, "fesom2_graph_launch")
    else if (mode == 4) then
      ! the rest of the host's uploads (ttf, fct_adf_v, fct_adf_h went up above), the pass, and
      ! del_ttf back into the host arrays on the same stream
      call transfer_var_async(h_lo, lo, s, no)
      call transfer_var_async(h_del_v, del_v, s, no)
      call transfer_var_async(h_del_h, del_h, s, no)
      call split_pass()
      call fesom2_transfer_back_async(h_del_v, del_v, s, istat); call check(istat, "fesom2_transfer_back_async")
      call fesom2_transfer_back_async(h_del_h, del_h, s, istat); call check(istat, "fesom2_transfer_back_async")
    else
      call split_pass()
    end if
    call await_stream(s, istat)
    call check(istat, "await_stream")
    call fesom2_download(h_plus, plus, istat); call fesom2_download(h_minus, minus, istat)
    call fesom2_download(h_adf_v, adf_v, istat); call fesom2_download(h_adf_h, adf_h, istat)
    if (mode /= 4) then
      call fesom2_download(h_del_v, del_v, istat); call fesom2_download(h_del_h, del_h, istat)
    end if
    call check(istat, "fesom2_download")
    if (mode == 2) call fesom2_graph_free(graph)
  end if

  open(newunit=u, file=trim(fout), access='stream', form='unformatted', status='replace')
  write(u) int(4, c_int64_t), st
  call write_ra(u, plus); call write_ra(u, minus); call write_ra(u, adf_v); call write_ra(u, adf_h)
  call write_ra(u, del_v); call write_ra(u, del_h)
  close(u)
  print '(a, 4i3, a, i3)', 'fct_ale_host: alg_state', st, '  tracers', ntr

contains

  ! the direction-split pass, device resident (fct_ale_pre_comm_v_acc_ -> fct_ale_post_comm_h_acc_)
  subroutine split_pass()
    call fct_ale_pre_comm_v_acc(st(1), s, ntr, h_plus, h_minus, h_ttf, h_lo, h_adf_v, h_adf_h, h_area_inv, h_area, &
        h_hnode, h_hnode_new, h_del_v, N, H, T, E, nl, h_nlev_nod, h_nlev_elem, h_elem_nodes, h_nie_num, h_nie, &
        dim, h_edges, h_edge_tri, vlimit, sc(2), sc(3), sc(1))
    call fct_ale_post_comm_h_acc(st(2), s, ntr, nullh, nullh, h_plus, h_minus, h_adf_h, h_del_h, h_area, &
        N, H, E, nl, h_nlev_nod, h_nlev_elem, h_edges, h_edge_tri, sc(1))
  end subroutine

  subroutine poison(handle, n)
    type(c_ptr) :: handle
    integer, intent(in) :: n
    real(c_double), allocatable :: junk(:)
    integer(c_int) :: istat
    allocate(junk(max(n, 1)))
    junk = 7.0_c_double
    call fesom2_upload(handle, junk, istat)
    call check(istat, "fesom2_upload")
    deallocate(junk)
  end subroutine

  subroutine check(istat, what)
    integer(c_int), intent(in) :: istat
    character(len=*), intent(in) :: what
    if (istat /= 0) then
      print *, 'fct_ale_host: ', what, ' failed, istat = ', istat
      error stop 2
    end if
  end subroutine

  subroutine upload_mesh(handle, a)
    type(c_ptr) :: handle
    integer(c_int), target :: a(:)
    integer(c_int) :: n, istat
    n = max(size(a), 1)
    call transfer_mesh(handle, a, n, istat)
    call check(istat, "transfer_mesh")
  end subroutine

  subroutine bind(handle, a, event)
    type(c_ptr) :: handle
    real(c_double), target :: a(:)
    logical(c_bool) :: event
    integer(c_int) :: n, istat
    n = size(a)
    call alloc_var(handle, a, n, event, istat)
    call check(istat, "alloc_var")
    call transfer_var(handle, a)
  end subroutine

  subroutine read_i(u, a)
    integer, intent(in) :: u
    integer(c_int), intent(out) :: a(:)
    integer(c_int64_t) :: n
    read(u) n
    if (n /= size(a)) error stop 3
    read(u) a
  end subroutine

  subroutine read_ia(u, a)
    integer, intent(in) :: u
    integer(c_int), allocatable, intent(out) :: a(:)
    integer(c_int64_t) :: n
    read(u) n
    allocate(a(n))
    if (n > 0) read(u) a
  end subroutine

  subroutine read_ra(u, a)
    integer, intent(in) :: u
    real(c_double), allocatable, intent(out) :: a(:)
    integer(c_int64_t) :: n
    read(u) n
    allocate(a(n))
    if (n > 0) read(u) a
  end subroutine

  subroutine write_ra(u, a)
    integer, intent(in) :: u
    real(c_double), intent(in) :: a(:)
    write(u) int(size(a), c_int64_t), a
  end subroutine
end program fct_ale_host
